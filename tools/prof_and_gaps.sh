set -u
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/gaps
MOVES=3 timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/gaps -o run --output-format csv -- python3 tools/gaps.py > gpurun_out/gaps/log.txt 2>&1 || exit $?
f=$(find gpurun_out/gaps -name "*kernel_trace.csv" | head -1); python3 tools/kt_gaps.py $f 60
bash tools/profile.sh
