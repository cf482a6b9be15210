"""Idle time between consecutive kernels of one rocprofv3 results db (kernel trace): span, busy, gap total, and the
gaps grouped by the kernel that follows them. Only dispatches after the first `skip` seconds of the trace count.
Usage: python tools/gaps.py gpurun_out/prof_x/<name>_results.db [last_ms]"""
import sqlite3
import sys
from collections import defaultdict

c = sqlite3.connect(sys.argv[1])
last_ms = float(sys.argv[2]) if len(sys.argv) > 2 else 50.0
rows = list(c.execute("""select d.start, d.end, s.display_name from rocpd_kernel_dispatch d
                         join rocpd_info_kernel_symbol s on d.kernel_id = s.id order by d.start"""))
t_end = rows[-1][1]
rows = [r for r in rows if r[0] >= t_end - last_ms * 1e6]
span = rows[-1][1] - rows[0][0]
busy = sum(r[1] - r[0] for r in rows)
gaps = defaultdict(list)
overlap = 0
for a, b in zip(rows, rows[1:]):
    g = b[0] - a[1]
    if g < 0:
        overlap += 1
    gaps[b[2].split("(")[0][:70]].append(max(g, 0))
print(f"window {span / 1e6:.3f} ms, {len(rows)} kernels, busy {busy / 1e6:.3f} ms ({100 * busy / span:.1f}%), "
      f"gaps {(span - busy) / 1e6:.3f} ms, overlapping starts {overlap}")
for name, gs in sorted(gaps.items(), key=lambda kv: -sum(kv[1])):
    gs.sort()
    print(f"{sum(gs) / 1e3:9.1f}us n={len(gs):5d} median {gs[len(gs) // 2] / 1e3:6.2f}us  before {name}")
