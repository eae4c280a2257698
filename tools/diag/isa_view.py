"""Compile geot_kernels.hip to gfx950 assembly with extra -D defines and print, per kernel, the
register/scratch use and a one-letter instruction-class trace of each basic block (M mfma, D ds,
G vmem, w waitcnt, B barrier, v valu, s salu): where the waits sit relative to the MFMAs.
usage: python tools/diag/isa_view.py [-DNAME=V ...] [--kernel REGEX] [--trace]"""
import os
import re
import subprocess
import sys

R = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
defs = [a for a in sys.argv[1:] if a.startswith("-D")]
kre = re.compile(sys.argv[sys.argv.index("--kernel") + 1] if "--kernel" in sys.argv else r"k_edge_layerINS_5BF16TELi0E")
out = "/tmp/isa_view.s"
subprocess.run(["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "--offload-arch=gfx950", "--offload-device-only", "-S",
                f"-I{R}/include", *defs, f"{R}/deepinteract_amd/csrc/geot_kernels.hip", "-o", out], check=True,
               stderr=subprocess.DEVNULL)
s = open(out).read()


def cls(op):
    if op.startswith("v_mfma"):
        return "M"
    if op.startswith("ds_"):
        return "D"
    if op.startswith(("buffer", "global")):
        return "G"
    if op.startswith("s_waitcnt"):
        return "w"
    if op.startswith("s_barrier"):
        return "B"
    if op.startswith("v_"):
        return "v"
    if op.startswith("s_"):
        return "s"
    return ""


for m in re.finditer(r"^(_ZN2di\w+):", s, re.M):
    name = m.group(1)
    if not kre.search(name):
        continue
    body = s[m.end():s.find("s_endpgm", m.end())]
    meta_at = s.find(".end_amdhsa_kernel", m.end())
    meta = s[s.rfind(".amdhsa_kernel " + name, 0, meta_at + 1):meta_at]
    g = {k: re.search(rf"\.amdhsa_{k}\s+(\d+)", meta) for k in ("next_free_vgpr", "accum_offset", "private_segment_fixed_size")}
    ops = [ln.split()[0] for ln in body.split("\n") if ln.strip() and not ln.strip().startswith((";", "."))]
    print(name, {k: int(v.group(1)) for k, v in g.items() if v}, "mfma", sum(o.startswith("v_mfma") for o in ops),
          "waitcnt", sum(o == "s_waitcnt" for o in ops), "scratch", sum("scratch" in o for o in ops))
    if "--trace" in sys.argv:
        for blk in re.split(r"\n(?=\.LBB)", body):
            t = "".join(cls(ln.split()[0]) for ln in blk.split("\n")[1:] if ln.strip() and not ln.strip().startswith((";", ".")))
            if "M" in t:
                print("  ", blk.split(":")[0][:10], t)
