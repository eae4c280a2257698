"""Where the chunked contact-map gather's extra time goes at world size 1 (verdict
item 7): predict_sharded over 4 C4 complexes (micro-batches of one) with gather none / chunked / once,
each 5 times interleaved; for the chunked runs the host time inside ChunkedGather.__init__, put()
and finish() and inside the forward calls, with and without a device synchronisation after every
micro-batch.

usage (GPU box): python tools/diag/gather_probe.py [--record [--extra-streams N] [--compute-stream] [--lib variant.so]]
(--record: bench.py's allgather_record alone in a fresh process, to compare with the same record
taken after the bench's timed steps)
"""
import json
import os
import sys
import time

import torch
import torch.distributed as dist

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from deepinteract_amd import distributed as D, synth  # noqa: E402
from deepinteract_amd.modules import LitGINI  # noqa: E402
from deepinteract_amd.weights import seeded_state_dict  # noqa: E402


def record():
    """bench.py's own allgather_record, in a fresh process (no bench run before it)."""
    if "--lib" in sys.argv:  # an A/B build (tools/diag/patch_build.py)
        from deepinteract_amd import _lib
        _lib.load_variant(sys.argv[sys.argv.index("--lib") + 1])
    import bench
    ws, rank, local = bench.dist_setup(force=True)
    dev = torch.device("cuda", local)
    extra = int(sys.argv[sys.argv.index("--extra-streams") + 1]) if "--extra-streams" in sys.argv else 0
    keep = [torch.cuda.Stream(dev) for _ in range(extra)]  # each one takes a hardware queue slot
    for s in keep:
        with torch.cuda.stream(s):
            torch.zeros(1, device=dev).add_(1)
    torch.cuda.synchronize()
    if "--compute-stream" in sys.argv:  # the whole record on a pool stream instead of the null stream
        with torch.cuda.stream(torch.cuda.Stream(dev)):
            r = bench.allgather_record(ws, rank, 256, 1000, 20, dev)
    else:
        r = bench.allgather_record(ws, rank, 256, 1000, 20, dev)
    print(json.dumps({"record_in_fresh_process": r["predict_sharded"], "extra_streams": extra,
                      "compute_stream": "--compute-stream" in sys.argv,
                      "GPU_MAX_HW_QUEUES": os.environ.get("GPU_MAX_HW_QUEUES")}))


def main():
    if "--record" in sys.argv:
        return record()
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", "29533")
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=dev)
    model = LitGINI(dtype="bf16", head_dtype=torch.bfloat16).to(dev).eval()
    model.load_reference_state_dict(seeded_state_dict(0))
    cx = [synth.synthetic_complex(50_000 + i, 1000, 1000) for i in range(4)]
    fwd = D.gpu_forward(model, 20)
    D.predict_sharded(cx[:1], fwd, micro_batch=1, dtype=torch.float32, device=dev, gather="none")

    acc = {}

    def timed_method(cls, name):
        orig = getattr(cls, name)

        def wrap(self, *a, **k):
            t0 = time.perf_counter()
            out = orig(self, *a, **k)
            acc[name] = acc.get(name, 0.0) + time.perf_counter() - t0
            return out
        setattr(cls, name, wrap)

    for n in ("__init__", "put", "finish", "slots"):
        timed_method(D.ChunkedGather, n)

    def fwd_timed(batch, ids, out=None):
        t0 = time.perf_counter()
        r = fwd(batch, ids, out=out) if out is not None else fwd(batch, ids)
        acc["forward"] = acc.get("forward", 0.0) + time.perf_counter() - t0
        return r

    def run(mode, f):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        D.predict_sharded(cx, f, micro_batch=1, dtype=torch.float32, device=dev, gather=mode)
        torch.cuda.synchronize()
        return time.perf_counter() - t0

    best = {}
    for _ in range(5):
        for mode in ("none", "chunked", "once"):
            acc.clear()
            t = run(mode, fwd_timed)
            if mode not in best or t < best[mode][0]:
                best[mode] = (t, dict(acc))
    for mode, (t, parts) in best.items():
        print(json.dumps({"mode": mode, "s": round(t, 4), "host_s": {k: round(v, 4) for k, v in parts.items()}}))
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
