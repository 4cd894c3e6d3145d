#!/bin/bash
# r03 combined: bin-mean parity + host copy rates + off-shape shapes (r03_seg.sh),
# then the medoid A/B and medoid tests (r03_md.sh).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$PWD}
cd "$R"
bash tools/gpu/r03_seg.sh || exit 1
VARIANTS="${VARIANTS:-mdbase main}" bash tools/gpu/r03_md.sh || exit 1
