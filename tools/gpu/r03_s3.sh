#!/bin/bash
# r03 session 2, call 2: medoid A/B ($VARIANTS) on configs[4], then the off-shape PMC.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$PWD}
cd "$R"
mkdir -p gpurun_out
VARIANTS="${VARIANTS:-base ilv base ilv}" WHICH=md CLUSTERS=385000 REPS=10 bash tools/gpu/ab.sh || exit 1
bash tools/gpu/shapes_pmc.sh
