"""Per-(kernel, grid) dispatch statistics from a rocprofv3 rocpd database: separates launches of
one kernel on different shapes (e.g. spatial vs temporal attention).
usage: python tools/rocprof_grid.py <results.db> <kernel-substring> [steps]"""
import collections
import sqlite3
import sys


def main():
    db = sqlite3.connect(sys.argv[1])
    sub = sys.argv[2]
    steps = float(sys.argv[3]) if len(sys.argv) > 3 else 1.0
    names = {r[0]: r[1] for r in db.execute('select id, display_name from rocpd_info_kernel_symbol')}
    agg = collections.defaultdict(list)
    q = ('select kernel_id, grid_size_x, grid_size_y, grid_size_z, workgroup_size_x, start, end '
         'from rocpd_kernel_dispatch')
    for kid, gx, gy, gz, wx, s, e in db.execute(q):
        n = names.get(kid, '?')
        if sub in n:
            agg[(n[:60], gx, gy, gz, wx)].append((e - s) / 1e3)
    print(f'{"kernel":60s} {"grid":>22s} {"wg":>5s} {"calls":>6s} {"avg_us":>9s} {"ms/step":>8s}')
    for (n, gx, gy, gz, wx), d in sorted(agg.items(), key=lambda kv: -sum(kv[1])):
        print(f'{n:60s} {f"{gx}x{gy}x{gz}":>22s} {wx:5d} {len(d):6d} {sum(d) / len(d):9.1f} '
              f'{sum(d) / 1e3 / steps:8.3f}')


if __name__ == '__main__':
    main()
