"""One-screen summary of a bench.py JSON line: python tools/show_bench.py <file>"""
import json
import sys


def main(path):
    d = json.loads([ln for ln in open(path) if ln.startswith("{")][-1])
    print(d.get("value"), d.get("ms_per_step"), "ranks", d.get("ranks_seen"), d.get("kernels_us"))
    for k, v in (d.get("secondary") or {}).items():
        if not isinstance(v, dict):
            continue
        rf = v.get("roofline") or {}
        print(f"  {k}: value={v.get('value')} ranks={v.get('ranks_seen')} frac={rf.get('frac')} "
              f"ms={v.get('ms_per_step')} wall={v.get('bench_wall_s')} err={v.get('error')} "
              f"ovl={(v.get('config') or {}).get('overlap_ranges')} e2e={(v.get('end_to_end') or {}).get('value')}")


if __name__ == "__main__":
    main(sys.argv[1])
