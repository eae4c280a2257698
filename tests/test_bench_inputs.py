"""bench.py's committed inputs reach the GPU box: the roofline's `traffic` field is read from
profiles/pmc_traffic.json at run time, so no .gpurunignore pattern may drop that file from the
snapshot the box (and the round-end driver) runs, and the pair stream's entry scales to a launch."""
import fnmatch
import json
import os

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
TRAFFIC = "profiles/pmc_traffic.json"


def _ignored(rel, patterns):
    """tar --exclude semantics as gpurun documents them: './x' anchors at the top, a bare pattern
    matches at any depth (any trailing part of the path), directories exclude their contents."""
    parts = rel.split("/")
    prefixes = ["/".join(parts[:i]) for i in range(1, len(parts) + 1)]
    for p in patterns:
        if p.startswith("./"):
            if any(fnmatch.fnmatch(x, p[2:]) for x in prefixes):
                return True
        elif any(fnmatch.fnmatch("/".join(parts[i:j]), p) for i in range(len(parts))
                 for j in range(i + 1, len(parts) + 1)):
            return True
    return False


def test_pmc_traffic_travels_to_the_gpu_box():
    path = os.path.join(ROOT, ".gpurunignore")
    patterns = [ln.strip() for ln in open(path) if ln.strip() and not ln.startswith("#")] if os.path.exists(path) else []
    assert not _ignored(TRAFFIC, patterns), f"{TRAFFIC} excluded by .gpurunignore: {patterns}"
    assert _ignored("profiles/r5_end_kernel_stats.csv", ["./profiles/*.csv"])  # the matcher itself
    assert _ignored("profiles/x.json", ["./profiles"])


def test_pair_traffic_scales_to_the_launch():
    import bench
    rec = json.load(open(os.path.join(ROOT, TRAFFIC)))["pair_tensor"]
    alg = 4.096e9 * 128
    assert bench.load_pmc_traffic("pair_tensor", alg) == rec["hbm_bytes_per_alg_byte"] * alg
    assert 1.0 <= rec["hbm_bytes_per_alg_byte"] < 1.1
    assert bench.load_pmc_traffic("pair_tensor") is None
    assert bench.load_pmc_traffic("edge_layer") > 0
