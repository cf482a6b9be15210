# GPU box: the named GPU test files (default: all), one pytest process. bash tools/gpu_tests.sh <tag> [files...]
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
T=${1:-r03}
shift || true
FILES=${@:-tests}
timeout -k 10 600 python -u -m pytest $FILES -m gpu -x -v --timeout 180 --timeout-method thread > gpurun_out/${T}_gpu_tests.log 2>&1 || { tail -60 gpurun_out/${T}_gpu_tests.log; exit 1; }
tail -3 gpurun_out/${T}_gpu_tests.log
