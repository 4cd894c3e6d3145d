#!/bin/bash
# PMC traffic passes first (bin-mean / medoid HBM bytes into profiles/pmc_traffic.json
# of this box's copy, so the bench line's roofline.traffic is this build's), then round.sh.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$PWD}
cd "$R"
bash tools/gpu/pmc.sh > gpurun_out/pmc_run.log 2>&1 || { tail -20 gpurun_out/pmc_run.log; exit 1; }
python3 - <<'PY' || exit 1
import json
new = json.load(open("gpurun_out/pmc/pmc_traffic.json"))
cur = json.load(open("profiles/pmc_traffic.json"))
for k, v in new.items():
    if not k.startswith("_"):
        cur[k] = v
json.dump(cur, open("profiles/pmc_traffic.json", "w"), indent=1)
json.dump(cur, open("gpurun_out/pmc_traffic_merged.json", "w"), indent=1)
print("traffic", {k: v for k, v in cur.items() if not k.startswith("_")})
PY
bash tools/gpu/round.sh
