#!/bin/bash
# Round-2 measurement pass on the GPU box: counter list, ResNet parity tests,
# the default bench line, MFMA busy + clock (bench workload), and SQ stall
# attribution of k_resnet (standalone, 4096 rows). Each step time-limited;
# stops at the first failure.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 60 rocprofv3 -L > gpurun_out/counters_list.txt 2>&1 || echo "counter list rc=$?"
timeout -k 10 300 python -m pytest tests/test_gpu_resnet.py tests/test_gpu_configs.py -m gpu -q --timeout 200 > gpurun_out/r02_tests.log 2>&1 || { tail -30 gpurun_out/r02_tests.log; exit 1; }
tail -3 gpurun_out/r02_tests.log
timeout -k 10 300 python bench.py --cpu-baseline-seconds 2 > gpurun_out/r02_bench.log 2>&1 || { tail -20 gpurun_out/r02_bench.log; exit 1; }
tail -1 gpurun_out/r02_bench.log
MFMA_TAG=${TAG:-r02_a} bash tools/mfma_pmc.sh || exit 1
ROWS=4096 NN_PMC_4="SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE" bash tools/nn_pmc.sh || exit 1
