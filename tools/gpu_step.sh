set -e
mkdir -p gpurun_out
export TMPDIR=/tmp
rm -rf gpurun_out/prof_fcl
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_fcl -o fcl -- python bench.py --workload fc_large --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/fcl_prof.log 2>&1
