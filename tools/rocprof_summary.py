"""Summarise a rocprofv3 --kernel-trace --stats database (rocpd sqlite) into a per-kernel table.
usage: python tools/rocprof_summary.py <results.db> [steps]"""
import re
import sqlite3
import sys


def short(name):
    name = re.sub(r'\(anonymous namespace\)::', '', name)
    name = re.sub(r'at::native::', '', name)
    m = re.match(r'(void )?([\w:<>, ]+?)\(', name)
    n = m.group(2) if m else name[:60]
    return n[:70]


def main():
    db = sqlite3.connect(sys.argv[1])
    steps = float(sys.argv[2]) if len(sys.argv) > 2 else 1.0
    rows = db.execute('select name, total_calls, total_duration, average, percentage from top_kernels').fetchall()
    total = sum(r[2] for r in rows)
    print(f'{"kernel":72s} {"calls":>7s} {"total_ms":>10s} {"avg_us":>9s} {"%":>6s}')
    for name, calls, tot, avg, pct in rows:
        print(f'{short(name):72s} {calls:7d} {tot / 1e3:10.3f} {avg:9.2f} {pct:6.2f}')
    print(f'{"TOTAL":72s} {"":7s} {total / 1e3:10.3f}   (per step: {total / 1e3 / steps:.2f} ms over {steps:g} profiled steps incl. warmup)')


if __name__ == '__main__':
    main()
