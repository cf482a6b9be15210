set -e
mkdir -p gpurun_out
for v in new old new old new old; do BCNF_AMD_LIB=build_exp/lib$v.so timeout -k 10 200 python bench.py --no-cpu-baseline --no-secondary > gpurun_out/b_$v.json 2>&1; echo $v $(tail -1 gpurun_out/b_$v.json | cut -c100-130); done
