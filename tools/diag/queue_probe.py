"""Which stream pairs of this process run concurrently (reach the GPU through different hardware
queues)? The evidence behind DESIGN.md §6 "hardware queues" (round 6).

usage (GPU box): python tools/diag/queue_probe.py [--nccl]
With --nccl a world-size-1 RCCL group is created first (bench.py --dist / torchrun), as the
communicator's own streams change which hardware queue later streams get. Prints one JSON line:
for each pair (waiter, signaller) whether a kernel on the signaller's stream ran while the waiter's
kernel was still waiting (di_streams_concurrent, 200 ms patience).
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from deepinteract_amd.pipeline import schedule_streams, streams_concurrent  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--nccl", action="store_true")
    ap.add_argument("--pool", type=int, default=4, help="torch pool streams to probe against the NULL stream")
    args = ap.parse_args()
    torch.cuda.set_device(0)
    out = {"nccl": args.nccl, "GPU_MAX_HW_QUEUES": os.environ.get("GPU_MAX_HW_QUEUES")}
    if args.nccl:
        import torch.distributed as dist
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", "29533")
        dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
        dist.barrier()
    null = torch.cuda.current_stream()
    pool = [torch.cuda.Stream() for _ in range(args.pool)]
    # round 5's bench pair: the pair stream (first pool stream) waits, the NULL (GeoT) stream signals
    out["pool_i_waits_null_signals"] = [streams_concurrent(p, null) for p in pool]
    out["pool_i_waits_pool_0_signals"] = [streams_concurrent(p, pool[0]) for p in pool[1:]]
    g, p = schedule_streams()
    out["dedicated_pair_waits_geot_signals"] = streams_concurrent(p, g)
    out["dedicated_geot_waits_pair_signals"] = streams_concurrent(g, p)
    out["dedicated_pair_waits_null_signals"] = streams_concurrent(p, null)
    out["dedicated_pair_waits_pool_i_signals"] = [streams_concurrent(p, q) for q in pool]
    print(json.dumps(out), flush=True)
    if args.nccl:
        import torch.distributed as dist
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
