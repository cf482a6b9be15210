# GPU box, one call (round 6): STEPS selects what runs, in this order, each under its own limit, the chain stopping at
# the first failure.  tests = the full GPU suite; testsf = the files in $TESTFILES (-k $TESTK when set); bench = the
# default bench line; rawab = device times of the folded training pass, working tree vs each of $AB_LIBS, three
# alternations; stamps = the phase stamps of the diagnostic builds in $STAMP_LIBS; prof = rocprofv3 kernel stats of
# the default bench; abbench = bench.py --no-secondary, working tree vs $AB_LIBS, $NABB (2) alternations; sampleab =
# the sampling bench line, working tree vs $AB_LIBS, two alternations.
#   bash tools/gpu_r06.sh <tag> "testsf rawab"
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
T=${1:-r06}
STEPS=${2:-"tests bench"}
PYT="python -u -m pytest -x -q --timeout 120 --timeout-method thread"
for s in $STEPS; do
  case $s in
    tests)
      timeout -k 10 600 $PYT tests -m gpu > gpurun_out/${T}_gpu_tests.log 2>&1 || { tail -40 gpurun_out/${T}_gpu_tests.log; exit 1; }
      tail -2 gpurun_out/${T}_gpu_tests.log ;;
    testsf)
      timeout -k 10 500 $PYT $TESTFILES -m gpu ${TESTK:+-k "$TESTK"} > gpurun_out/${T}_gpu_testsf.log 2>&1 || { tail -40 gpurun_out/${T}_gpu_testsf.log; exit 1; }
      tail -2 gpurun_out/${T}_gpu_testsf.log ;;
    bench)
      timeout -k 10 420 python bench.py > gpurun_out/${T}_bench.json 2> gpurun_out/${T}_bench.err || { tail -20 gpurun_out/${T}_bench.err; exit 1; }
      python tools/show_bench.py gpurun_out/${T}_bench.json ;;
    rawab)
      for i in $(seq 1 ${NALT:-3}); do
        timeout -k 10 120 python tools/raw_probe.py
        for lib in ${AB_LIBS:-build_exp/libhead.so}; do BCNF_AMD_LIB=$lib timeout -k 10 120 python tools/raw_probe.py; done
      done 2>&1 | grep -v amdgpu.ids | tee gpurun_out/${T}_rawab.txt ;;
    stamps)
      for i in 1 2; do
        for lib in ${STAMP_LIBS:-build_exp/libstamps.so}; do BCNF_AMD_LIB=$lib timeout -k 10 120 python tools/raw_probe.py; done
      done 2>&1 | grep -v amdgpu.ids | tee gpurun_out/${T}_stamps.txt ;;
    abbench)
      for i in $(seq 1 ${NABB:-2}); do for lib in default ${AB_LIBS:-build_exp/libhead.so}; do
        if [ $lib = default ]; then timeout -k 10 200 python bench.py --no-secondary --no-cpu-baseline $ABARGS > gpurun_out/${T}_abb.json 2>/dev/null
        else BCNF_AMD_LIB=$lib timeout -k 10 200 python bench.py --no-secondary --no-cpu-baseline $ABARGS > gpurun_out/${T}_abb.json 2>/dev/null; fi
        python -c "import json; d=json.loads(open('gpurun_out/${T}_abb.json').read().strip().splitlines()[-1]); print('$lib', d['ms_per_step'], round(d['value']), d['kernels_us'])"
      done; done 2>&1 | tee gpurun_out/${T}_abbench.txt ;;
    sampleab)
      for i in 1 2; do for lib in default ${AB_LIBS:-build_exp/libhead.so}; do
        if [ $lib = default ]; then timeout -k 10 200 python bench.py --workload sample --no-cpu-baseline > gpurun_out/${T}_sab.json 2>/dev/null
        else BCNF_AMD_LIB=$lib timeout -k 10 200 python bench.py --workload sample --no-cpu-baseline > gpurun_out/${T}_sab.json 2>/dev/null; fi
        python -c "import json; d=json.loads(open('gpurun_out/${T}_sab.json').read().strip().splitlines()[-1]); print('$lib', d['ms_per_step'], round(d['value']))"
      done; done 2>&1 | tee gpurun_out/${T}_sampleab.txt ;;
    prof)
      bash tools/profile_round.sh $T > gpurun_out/${T}_prof.log 2>&1 || { tail -20 gpurun_out/${T}_prof.log; exit 1; }
      tail -5 gpurun_out/${T}_prof.log ;;
    *) echo "unknown step $s"; exit 1 ;;
  esac
done
