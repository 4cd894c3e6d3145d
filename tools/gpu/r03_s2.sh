#!/bin/bash
# r03 session 2: the round's evidence (full.sh), then an A/B of the medoid variants
# in $VARIANTS (specpride_amd/lib/ab_<v>.so) on the configs[4] batch.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$PWD}
cd "$R"
bash tools/gpu/full.sh || exit 1
VARIANTS="${VARIANTS:-base p3 p1 p13 base}" WHICH=md CLUSTERS=385000 REPS=10 bash tools/gpu/ab.sh
