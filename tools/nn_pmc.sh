#!/bin/bash
# SQ wave-state counters of k_resnet (standalone, tools/nn_ablation.py):
# WAIT_ANY = parked in s_waitcnt / barrier, WAIT_INST_ANY = issue-stalled,
# ACTIVE_INST_ANY = issuing (quad-cycles; disjoint, sum ~ WAVE_CYCLES).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/npmc
for set in "${NN_PMC_1:-SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY}" "${NN_PMC_2:-SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_MISC}" "${NN_PMC_3:-SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM}" ${NN_PMC_4:+"$NN_PMC_4"}; do
  d=gpurun_out/npmc/$(echo $set | cut -d' ' -f1)
  timeout -k 10 300 rocprofv3 --pmc $set -d $d -o run --output-format csv -- python3 tools/nn_ablation.py > $d.log 2>&1
  rc=$?; echo "pmc [$set] rc=$rc"; [ $rc -eq 0 ] || { tail -3 $d.log; exit $rc; }
done
python3 - <<'PY'
import csv, glob
from collections import defaultdict
acc = defaultdict(list)
for f in glob.glob("gpurun_out/npmc/**/run_counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if "k_resnet" in r["Kernel_Name"]:
            acc[r["Counter_Name"]].append(float(r["Counter_Value"]))
print({c: round(sum(v) / len(v)) for c, v in sorted(acc.items())})
PY
