# Diagnostic builds of the library (CPU container): bash tools/exp_variants.sh stamps [extra hipcc flags]
# -> build_exp/libstamps.so with the phase-stamp code (-DBCNF_PHASE_STAMPS: s_memtime per phase of workgroup 0,
# bcnf_debug_phases / bcnf_wide_debug_phases exports; tools/kbench.py, tools/link_phases.py read them). The shipped
# library (__graft_entry__.build) never contains this code. Results of a stamped build are valid; its timings are
# ~10% slow (each stamp waits for the scalar memory counter).
set -e
cd "$(dirname "$0")/.."
mkdir -p build_exp
name=${1:-stamps}
shift || true
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -shared -fPIC -Iinclude -DBCNF_PHASE_STAMPS "$@" \
  bcnf_amd/csrc/bcnf_stack.hip bcnf_amd/csrc/bcnf_train.hip bcnf_amd/csrc/bcnf_wide.hip bcnf_amd/csrc/bcnf_eval.hip bcnf_amd/csrc/bcnf_resim.hip \
  -o build_exp/lib$name.so
ls -la build_exp
