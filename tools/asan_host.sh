# AddressSanitizer run of the C-ABI's host code (SURVEY §5 "ASan-host on the C ABI"): the library built with
# -fsanitize=address on the HOST side only (device code unsanitized: GPU ASan is not available on this pool), loaded
# into the CPU tests that exercise the host arithmetic -- descriptor validation, layouts, parameter counts, workspace
# / slab / packed sizes, the pack-free forward's raw table, the wide backward's G-region plan at edge batches, the
# fold Adam spec. No GPU needed; run in the build container:  bash tools/asan_host.sh [log]
set -e
cd "$(dirname "$0")/.."
mkdir -p build_exp
LOG=${1:-profiles/r06_asan_host.txt}
RT=$(ls /opt/rocm/lib/llvm/lib/clang/*/lib/linux/libclang_rt.asan-x86_64.so | head -1)
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -shared -fPIC -Iinclude \
  -Xarch_host -fsanitize=address -Xarch_host -fno-omit-frame-pointer -Xarch_host -g \
  bcnf_amd/csrc/bcnf_stack.hip bcnf_amd/csrc/bcnf_train.hip bcnf_amd/csrc/bcnf_wide.hip bcnf_amd/csrc/bcnf_eval.hip \
  bcnf_amd/csrc/bcnf_resim.hip -o build_exp/libasan.so
nm -D build_exp/libasan.so | grep -c " U __asan_" | sed 's/^/asan runtime references in the library: /' > "$LOG"
{
  echo "runtime: $RT"
  LD_PRELOAD=$RT ASAN_OPTIONS=detect_leaks=0:halt_on_error=1:abort_on_error=1 BCNF_AMD_LIB=build_exp/libasan.so \
    python -m pytest tests/test_native_abi.py tests/test_configs_cpu.py tests/test_variants_cpu.py -m "not gpu" -q -p no:cacheprovider 2>&1
  echo "exit status: $?"
  # negative control: the same run must catch a host-side overflow -- the raw table written into a buffer 4 bytes
  # short (numpy's allocation goes through the ASan malloc interceptor)
  echo "negative control (expected: heap-buffer-overflow, non-zero exit):"
  set +e
  LD_PRELOAD=$RT ASAN_OPTIONS=detect_leaks=0 BCNF_AMD_LIB=build_exp/libasan.so python - <<'PY' 2>&1 | grep -m1 -o "ERROR: AddressSanitizer: [a-z-]*"
import ctypes
import numpy as np
from bcnf_amd import _native as N
L = N.lib()
d = N.make_desc(19, [16] * 7, 32, 80, 0.383, True)
nb = ctypes.c_int64()
assert L.bcnf_fold_raw_table_bytes(ctypes.byref(d), 90, ctypes.byref(nb)) == N.OK
buf = np.empty(nb.value - 4, np.uint8)
L.bcnf_fold_raw_table(ctypes.byref(d), 90, ctypes.c_void_p(buf.ctypes.data))
print("not caught")
PY
  echo "control exit status: ${PIPESTATUS[0]}"
  set -e
} >> "$LOG" 2>&1
tail -4 "$LOG"
