#!/bin/bash
# A/B of ab_old.so vs ab_new.so on the configs[4] batch (bin-mean, medoid), twice each.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$PWD}
cd "$R"
mkdir -p gpurun_out
VARIANTS="old new old new" WHICH=bm,md CLUSTERS=385000 REPS=10 bash tools/gpu/ab.sh
