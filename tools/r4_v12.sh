#!/bin/bash
# round 4 v12: 2 (default) / 3 / 4 GeoT workspace slots (3 rounds): with 2 slots GeoT(m+1) waits for
# pair(m-1) at every micro-batch boundary (profiles/r4_timeline.txt: 49 us GeoT-stream gap per micro-batch)
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"; cd "$R"
tools/ab.sh 3 "s2|" "s3|--slots 3" "s4|--slots 4"
