"""RCCL probe on one GPU: world_size ranks share cuda:0 and run the all_to_all_single that
noahgameframe_amd/shard.py's migration uses (int64 rows, uneven splits).  Exits non-zero on any
mismatch.  torchrun --nproc-per-node 2 tools/rccl_probe.py"""
import os

import torch
import torch.distributed as dist


def main():
    rank, ws = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    torch.cuda.set_device(0)
    dist.init_process_group("nccl", device_id=torch.device("cuda", 0))
    rw = 7
    scount = [(rank + d) % 3 + 1 for d in range(ws)]          # rows to each destination
    rcount = [(s + rank) % 3 + 1 for s in range(ws)]          # rows from each source
    sbuf = torch.empty((sum(scount), rw), dtype=torch.int64, device="cuda")
    at = 0
    for dst in range(ws):
        for i in range(scount[dst]):
            sbuf[at] = torch.arange(rw, device="cuda") + 1000 * rank + 100 * dst + 10 * i
            at += 1
    rbuf = torch.empty((sum(rcount), rw), dtype=torch.int64, device="cuda")
    dist.all_to_all_single(rbuf.view(-1), sbuf.view(-1), [c * rw for c in rcount], [c * rw for c in scount])
    torch.cuda.synchronize()
    at = 0
    for src in range(ws):
        for i in range(rcount[src]):
            want = torch.arange(rw, device="cuda") + 1000 * src + 100 * rank + 10 * i
            assert torch.equal(rbuf[at], want), (rank, src, i, rbuf[at].tolist())
            at += 1
    dist.barrier()
    if rank == 0:
        print("rccl all_to_all_single ok", ws)
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
