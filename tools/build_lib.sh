# Plain (shipped-flags) build of the library under another name, for same-box A/B runs: bash tools/build_lib.sh head
set -e
cd "$(dirname "$0")/.."
mkdir -p build_exp
name=${1:-head}
shift || true
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -shared -fPIC -Iinclude "$@" \
  bcnf_amd/csrc/bcnf_stack.hip bcnf_amd/csrc/bcnf_train.hip bcnf_amd/csrc/bcnf_wide.hip bcnf_amd/csrc/bcnf_eval.hip \
  bcnf_amd/csrc/bcnf_resim.hip -o build_exp/lib$name.so
