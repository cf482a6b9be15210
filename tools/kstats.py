"""Per-kernel summary of one rocprofv3 results db: calls, avg us, total ms, grid (first dispatch).
Usage: python tools/kstats.py gpurun_out/prof_x/<name>_results.db [top]"""
import sqlite3
import sys

c = sqlite3.connect(sys.argv[1])
top = int(sys.argv[2]) if len(sys.argv) > 2 else 30
q = """select s.display_name, count(*), avg(d.end-d.start), sum(d.end-d.start), min(d.grid_size_x), min(d.grid_size_y),
       min(d.grid_size_z), min(d.workgroup_size_x)
       from rocpd_kernel_dispatch d join rocpd_info_kernel_symbol s on d.kernel_id=s.id group by s.display_name
       order by sum(d.end-d.start) desc"""
rows = list(c.execute(q))
tot = sum(r[3] for r in rows)
for r in rows[:top]:
    print(f"{r[3] / 1e6:9.2f}ms {r[1]:6d} {r[2] / 1e3:9.1f}us {100 * r[3] / tot:5.1f}% grid=({r[4]},{r[5]},{r[6]}) "
          f"wg={r[7]} {r[0][:110]}")
