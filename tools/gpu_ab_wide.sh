# GPU box: wide GPU tests, then same-box A/B of FC_large / LSTM_large: working tree vs build_exp/libhead.so
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
T=${1:-r03}
timeout -k 10 300 python -u -m pytest tests/test_gpu_wide.py tests/test_gpu_configs.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/${T}_wide_tests.log 2>&1 || { tail -40 gpurun_out/${T}_wide_tests.log; exit 1; }
tail -1 gpurun_out/${T}_wide_tests.log
bash tools/ab_wide.sh fc_large build_exp/libhead.so 2>&1 | tee gpurun_out/${T}_ab_fc_large.txt
bash tools/ab_wide.sh lstm_large build_exp/libhead.so 2>&1 | tee gpurun_out/${T}_ab_lstm_large.txt
