"""Regenerate tools/sessions/INDEX.md from the header comment of every GPU session script.
usage: python tools/session_index.py"""
import os
import re

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
D = os.path.join(ROOT, "tools", "sessions")
HEADER = """# GPU session scripts

One script per `gpurun` call that produced a record cited in `DESIGN.md` §8: `g*.sh` are round 5's
(§8 "Round 5"), `r6_*.sh` round 6's (§8 "Round 6"). Each runs on the GPU box from the repository
root and writes under `gpurun_out/`; the summaries that DESIGN cites are copied into `profiles/`.
Variant and diagnostic libraries they load are built on the CPU first
(`tools/build_variants.py`, `tools/diag/patch_build.py <name>`, `tools/diag/build_rev.py`). The
reusable runners are `tools/ab.sh` (interleaved A/B of bench configurations) and
`tools/prof_round.sh` (end-of-round suite, bench lines and rocprofv3 passes). Regenerate this file
with `python tools/session_index.py`.

| script | what it measured (its header) |
|---|---|
"""


def key(f):
    m = re.match(r"(g|r6_)(\d+)", f)
    return (0 if f.startswith("g") else 1, int(m.group(2)) if m else 0, f)


def main():
    rows = []
    for f in sorted((f for f in os.listdir(D) if f.endswith(".sh")), key=key):
        lines = [ln[2:].strip() for ln in open(os.path.join(D, f)) if ln.startswith("# ")]
        desc = " ".join(lines[:2]) if lines else "(command record, no header: round 5 parity + bench of the pair queue)"
        desc = re.sub(r"\s+", " ", desc).replace("|", "/")
        rows.append(f"| `{f}` | {desc} |")
    with open(os.path.join(D, "INDEX.md"), "w") as fh:
        fh.write(HEADER + "\n".join(rows) + "\n")
    print(len(rows), "scripts")


if __name__ == "__main__":
    main()
