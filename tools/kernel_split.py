"""Split a rocprofv3 --stats kernel summary (kernel_stats.csv) into what runs where: the library's own HIP kernels
(bcnf_*.hip, anonymous-namespace k_*), MIOpen's LSTM (LSTM*HidUpdate and the tensor / reduce / copy kernels of its
RNN path), rocBLAS / hipBLASLt GEMMs (Cijk_*: issued by MIOpen's LSTM and by torch), and other ATen kernels.
python tools/kernel_split.py profiles/<run>_kernel_stats.csv [steps]   (steps: divide totals by it)"""
import csv
import sys
from collections import defaultdict

MIOPEN = ("LSTM", "Op2dTensor", "SubTensorOp", "gridwise_generic_reduce", "Op1dTensor", "Op3dTensor", "Op4dTensor",
          "MIOpen", "miopen", "ScaleTensor", "SetTensor", "CopyTensor", "transpose", "Transpose")


def category(name):
    if name.startswith("void (anonymous namespace)::k_") or name.startswith("(anonymous namespace)::k_"):
        return "bcnf_amd HIP kernels"
    if name.startswith("Cijk_"):
        return "rocBLAS/hipBLASLt GEMMs (MIOpen LSTM gates, torch)"
    if any(k in name for k in MIOPEN):
        return "MIOpen LSTM (cell updates, tensor ops, reduces)"
    if "copyBuffer" in name or "fillBuffer" in name:
        return "HIP runtime copies / fills"
    return "other ATen kernels (dropout, cat, elementwise)"


def main(path, steps=1.0):
    tot = defaultdict(float)
    top = defaultdict(list)
    for row in csv.DictReader(open(path)):
        c = category(row["Name"])
        ns = float(row["TotalDurationNs"])
        tot[c] += ns
        top[c].append((ns, row["Name"][:90], int(row["Calls"])))
    all_ns = sum(tot.values())
    for c, ns in sorted(tot.items(), key=lambda kv: -kv[1]):
        print(f"{c:55s} {ns / steps / 1e6:9.3f} ms  {100 * ns / all_ns:5.1f}%")
        for t, n, calls in sorted(top[c], reverse=True)[:4]:
            print(f"    {t / steps / 1e6:8.3f} ms  {calls:6d} calls  {n}")
    print(f"{'total':55s} {all_ns / steps / 1e6:9.3f} ms")


if __name__ == "__main__":
    main(sys.argv[1], float(sys.argv[2]) if len(sys.argv) > 2 else 1.0)
