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


def test_gpus_flag_starts_the_ranks(tmp_path):
    """`bench.py --gpus N` without a launcher starts N rank processes with the launcher's
    environment (RANK, LOCAL_RANK, WORLD_SIZE = N, rendezvous on 127.0.0.1); a launched rank
    whose WORLD_SIZE disagrees with --gpus refuses to run."""
    import json
    import pytest
    b = _bench()
    probe = tmp_path / "probe.py"
    probe.write_text("import json, os, sys\n"
                     "keys = ('RANK', 'LOCAL_RANK', 'WORLD_SIZE', 'MASTER_ADDR', 'MASTER_PORT')\n"
                     "open(sys.argv[1] + os.environ['RANK'], 'w').write(json.dumps({k: os.environ[k] for k in keys}))\n")
    assert b.spawn_ranks(3, [str(tmp_path / "r")], script=str(probe)) == 0
    seen = [json.loads((tmp_path / f"r{i}").read_text()) for i in range(3)]
    assert [s["RANK"] for s in seen] == ["0", "1", "2"] and [s["LOCAL_RANK"] for s in seen] == ["0", "1", "2"]
    assert {s["WORLD_SIZE"] for s in seen} == {"3"} and {s["MASTER_ADDR"] for s in seen} == {"127.0.0.1"}
    assert len({s["MASTER_PORT"] for s in seen}) == 1
    os.environ.pop("WORLD_SIZE", None)
    assert b.world_from_env(1) == (1, 0, 0)
    try:
        os.environ["WORLD_SIZE"] = "2"
        with pytest.raises(SystemExit):
            b.world_from_env(4)
    finally:
        os.environ.pop("WORLD_SIZE", None)


def test_a_failing_rank_stops_the_others(tmp_path):
    """If one rank fails, bench.py stops the others (by PID) and exits with that rank's code
    instead of waiting for a collective that can never complete."""
    import time
    b = _bench()
    probe = tmp_path / "probe.py"
    probe.write_text("import os, sys, time\n"
                     "if os.environ['RANK'] == '1':\n    sys.exit(3)\n"
                     "time.sleep(120)\n")
    t = time.time()
    assert b.spawn_ranks(2, [], script=str(probe)) == 3
    assert time.time() - t < 60
