# Build A/B experiment variants of the library (CPU container): bash tools/exp_variants.sh 1 2 4 8
set -e
cd "$(dirname "$0")/.."
mkdir -p build_exp
for e in "$@"; do
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -shared -fPIC -Iinclude -DBCNF_EXP=$e \
    bcnf_amd/csrc/bcnf_stack.hip bcnf_amd/csrc/bcnf_train.hip bcnf_amd/csrc/bcnf_wide.hip bcnf_amd/csrc/bcnf_eval.hip \
    -o build_exp/libexp$e.so &
done
wait
ls -la build_exp
