# GPU box, one call (round 5): STEPS selects what runs, in this order, each under its own limit, the chain stopping at
# the first failure:  tests = the full GPU suite; bench = the default bench line; bench2 = `bench.py --gpus 2` (two
# ranks sharing the card over gloo: a plumbing rehearsal, not a scaling number); abk = same-box A/B of the FC_small
# kernels against build_exp/libhead.so; abraw = the pack-free folded forward on / off (BCNF_FOLD_RAW); prof = rocprofv3 kernel stats of the default bench.
#   bash tools/gpu_r05.sh <tag> "tests bench bench2"
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
T=${1:-r04}
STEPS=${2:-"tests bench"}
for s in $STEPS; do
  case $s in
    probe)
      /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -shared -fPIC tools/probe_issue.hip -o /tmp/probe_issue.so 2>/dev/null || true
      [ -f tools/probe_issue.so ] || cp /tmp/probe_issue.so tools/probe_issue.so
      timeout -k 10 180 python tools/probe_issue.py ${PROBES:-} 2>&1 | grep -v amdgpu.ids | tee gpurun_out/${T}_probe.txt ;;
    rawab)   # device times of the folded training pass (pack-free forward) for the working tree and each AB_LIBS
      for i in 1 2 3; do
        timeout -k 10 120 python tools/raw_probe.py
        for lib in ${AB_LIBS:-build_exp/libhead.so}; do BCNF_AMD_LIB=$lib timeout -k 10 120 python tools/raw_probe.py; done
      done 2>&1 | grep -v amdgpu.ids | tee gpurun_out/${T}_rawab.txt ;;
    tests)
      timeout -k 10 540 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/${T}_gpu_tests.log 2>&1 || { tail -40 gpurun_out/${T}_gpu_tests.log; exit 1; }
      tail -2 gpurun_out/${T}_gpu_tests.log ;;
    testsf)   # the files in $TESTFILES
      timeout -k 10 400 python -u -m pytest $TESTFILES -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/${T}_gpu_testsf.log 2>&1 || { tail -40 gpurun_out/${T}_gpu_testsf.log; exit 1; }
      tail -2 gpurun_out/${T}_gpu_testsf.log ;;
    testsk)
      timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "$TESTK" > gpurun_out/${T}_gpu_testsk.log 2>&1 || { tail -40 gpurun_out/${T}_gpu_testsk.log; exit 1; }
      tail -2 gpurun_out/${T}_gpu_testsk.log ;;
    bench)
      timeout -k 10 420 python bench.py > gpurun_out/${T}_bench.json 2> gpurun_out/${T}_bench.err || { tail -20 gpurun_out/${T}_bench.err; exit 1; }
      python tools/show_bench.py gpurun_out/${T}_bench.json ;;
    bench2)
      timeout -k 10 420 python bench.py --gpus 2 --no-cpu-baseline > gpurun_out/${T}_bench2.json 2> gpurun_out/${T}_bench2.err || { tail -20 gpurun_out/${T}_bench2.err; exit 1; }
      python tools/show_bench.py gpurun_out/${T}_bench2.json ;;
    abk)
      for i in 1 2; do
        timeout -k 10 120 python tools/abk.py
        for lib in ${AB_LIBS:-build_exp/libhead.so}; do BCNF_AMD_LIB=$lib timeout -k 10 120 python tools/abk.py; done
      done 2>&1 | grep -v amdgpu.ids | tee gpurun_out/${T}_ab_kernels.txt ;;
    absample)
      bash tools/ab_sample.sh ${AB_LIBS:-build_exp/libhead.so} 2>&1 | tee gpurun_out/${T}_ab_sample.txt ;;
    pmc)
      bash tools/pmc_insts.sh $T > gpurun_out/${T}_pmc.log 2>&1 || { tail -20 gpurun_out/${T}_pmc.log; exit 1; }
      python tools/summarize_pmc.py $T | tail -30 ;;
    proflstm|proffcl)
      wl=$([ $s = proflstm ] && echo lstm_large || echo fc_large)
      cd /tmp && export TMPDIR=/tmp
      timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/${T}_$s -o run -- python3 $GRAFT_REPO_ROOT/bench.py --workload $wl --no-cpu-baseline --steps 10 --warmup 3 --kernel-iters 3 > $GRAFT_REPO_ROOT/gpurun_out/${T}_$s.log 2>&1 || { tail -20 $GRAFT_REPO_ROOT/gpurun_out/${T}_$s.log; exit 1; }
      cd $GRAFT_REPO_ROOT
      python tools/show_stats.py gpurun_out/${T}_$s 40 ;;
    lstmab)
      for i in 1 2; do for mi in 1 0; do
        BCNF_LSTM_MIOPEN=$mi timeout -k 10 200 python bench.py --workload lstm_large --no-cpu-baseline --steps 10 --warmup 3 > gpurun_out/${T}_lstmab.json 2>/dev/null
        python -c "import json; d=json.loads(open('gpurun_out/${T}_lstmab.json').read().strip().splitlines()[-1]); print('miopen=$mi', d['ms_per_step'], round(d['value']), d['kernels_us'])"
      done; done 2>&1 | tee gpurun_out/${T}_lstmab.txt ;;
    abbench)
      for i in 1 2; do for lib in default ${AB_LIBS:-build_exp/libhead.so}; do
        if [ $lib = default ]; then timeout -k 10 200 python bench.py --no-secondary --no-cpu-baseline > gpurun_out/${T}_abb.json 2>/dev/null
        else BCNF_AMD_LIB=$lib timeout -k 10 200 python bench.py --no-secondary --no-cpu-baseline > gpurun_out/${T}_abb.json 2>/dev/null; fi
        python -c "import json; d=json.loads(open('gpurun_out/${T}_abb.json').read().strip().splitlines()[-1]); print('$lib', d['ms_per_step'], round(d['value']), d['kernels_us'])"
      done; done 2>&1 | tee gpurun_out/${T}_abbench.txt ;;
    abwl)
      for i in 1 2; do for wl in ${WLS:-fc_large}; do for lib in ${AB_LIBS:-build_exp/libprev.so}; do
        BCNF_AMD_LIB=$lib timeout -k 10 200 python bench.py --workload $wl --no-secondary --no-cpu-baseline --steps 20 --warmup 5 > gpurun_out/${T}_abw.json 2>/dev/null
        python -c "import json; d=json.loads(open('gpurun_out/${T}_abw.json').read().strip().splitlines()[-1]); print('$wl $lib', d['ms_per_step'], round(d['value']), d.get('kernels_us'))"
      done; done; done 2>&1 | tee gpurun_out/${T}_abwl.txt ;;
    abunroll)   # r04zj only: the BCNF_EPOCH_UNROLL / BCNF_REMAINDER_GRAPH switches were a temporary build of train.py
      for i in 1 2; do for K in 20 50; do for cfg in "8 0" "8 1" "16 1"; do set -- $cfg
        BCNF_EPOCH_UNROLL=$1 BCNF_REMAINDER_GRAPH=$2 timeout -k 10 200 python bench.py --no-secondary --no-cpu-baseline --steps $K > gpurun_out/${T}_abu.json 2>/dev/null
        python -c "import json; d=json.loads(open('gpurun_out/${T}_abu.json').read().strip().splitlines()[-1]); print('K=$K unroll=$1 rem=$2', d['ms_per_step'], round(d['value']))"
      done; done; done 2>&1 | tee gpurun_out/${T}_abunroll.txt ;;
    abside)
      for i in 1 2; do for wl in fc_large lstm_large; do for sd in 1 0; do
        BCNF_WIDE_SIDE=$sd timeout -k 10 200 python bench.py --workload $wl --no-cpu-baseline --steps 20 --warmup 5 > gpurun_out/${T}_abs.json 2>/dev/null
        python -c "import json; d=json.loads(open('gpurun_out/${T}_abs.json').read().strip().splitlines()[-1]); print('$wl side=$sd', d['ms_per_step'], round(d['value']))"
      done; done; done 2>&1 | tee gpurun_out/${T}_abside.txt ;;
    abraw)
      for i in 1 2 3; do for raw in 1 0; do
        BCNF_FOLD_RAW=$raw timeout -k 10 200 python bench.py --no-secondary --no-cpu-baseline > gpurun_out/${T}_abr.json 2>/dev/null
        python -c "import json; d=json.loads(open('gpurun_out/${T}_abr.json').read().strip().splitlines()[-1]); print('raw=$raw', d['ms_per_step'], round(d['value']), d['kernels_us'])"
      done; done 2>&1 | tee gpurun_out/${T}_abraw.txt ;;
    prof)
      cd /tmp && export TMPDIR=/tmp
      timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/${T}_prof -o run -- python3 $GRAFT_REPO_ROOT/bench.py --no-secondary --no-cpu-baseline --steps 40 > $GRAFT_REPO_ROOT/gpurun_out/${T}_prof.log 2>&1 || { tail -20 $GRAFT_REPO_ROOT/gpurun_out/${T}_prof.log; exit 1; }
      cd $GRAFT_REPO_ROOT ;;
  esac
done
