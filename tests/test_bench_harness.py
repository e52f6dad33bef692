"""bench.py's own host bookkeeping (CPU): the migration harness's row queue."""
import importlib.util
import os

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _bench():
    spec = importlib.util.spec_from_file_location("nf_bench", os.path.join(ROOT, "bench.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def test_row_queue_is_fifo():
    """RowQueue.take / append against a plain list model: the oldest rows leave first, arrivals
    queue behind them, short takes return what is left, an empty queue returns None."""
    RowQueue = _bench().RowQueue
    rng = np.random.default_rng(5)
    start = np.arange(1000 * 5, dtype=np.int64).reshape(1000, 5)
    q, model, nxt = RowQueue(start), [tuple(r) for r in start], 10 ** 6
    for _ in range(300):
        if rng.random() < 0.5:
            k = int(rng.integers(0, 40))
            rows = np.arange(nxt, nxt + 5 * k, dtype=np.int64).reshape(k, 5)
            nxt += 5 * k
            q.append(rows)
            model += [tuple(r) for r in rows]
        else:
            n = int(rng.integers(1, 90))
            got = q.take(n)
            want, model = model[:n], model[n:]
            if not want:
                assert got is None
            else:
                assert [tuple(r) for r in got] == want
        assert len(q) == len(model)
    assert q.take(len(model) + 5) is not None or not model
    assert len(q) == 0 and q.take(3) is None
