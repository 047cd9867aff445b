"""Timeline of one contrastive step per stream from a rocprofv3 kernel trace (rocpd sqlite):
clusters of back-to-back kernels on each stream (split at idle gaps > gap_us), as offsets from the
step's first main-stream kernel, so the critical stream and its waits are visible.
usage: python tools/rocprof_timeline.py <results.db> [step_marker_substring] [gap_us]"""
import sqlite3
import sys


def short(n):
    n = n.replace('(anonymous namespace)::', '').replace('void ', '')
    return n.split('(')[0]


def main():
    db = sqlite3.connect(sys.argv[1])
    marker = sys.argv[2] if len(sys.argv) > 2 else 'patch_ln_strip'
    gap = float(sys.argv[3]) if len(sys.argv) > 3 else 150.0
    rows = sorted(db.execute('select start, "end", stream_id, name from kernels').fetchall())
    starts = [r[0] for r in rows if marker in r[3]]
    if len(starts) < 3:
        print('fewer than 3 step markers'); return
    t0, t1 = starts[-2], starts[-1]          # the last complete step
    print(f'step {1e-6 * (t1 - t0):.2f} ms (marker {marker})')
    step = [r for r in rows if t0 <= r[0] < t1]
    for q in sorted({r[2] for r in step}):
        seq = [r for r in step if r[2] == q]
        busy = sum(e - s for s, e, _, _ in seq)
        print(f'stream {q}: {len(seq)} kernels, kernel time {busy / 1e6:.2f} ms')
        cl = []
        for s, e, _, n in seq:
            if cl and s - cl[-1][1] <= gap * 1e3:
                c = cl[-1]
                c[1] = max(c[1], e); c[2] += 1; c[3] += e - s; c[5] = n
            else:
                cl.append([s, e, 1, e - s, n, n])
        for s, e, k, b, a, z in cl:
            print(f'  {1e-6 * (s - t0):7.2f} .. {1e-6 * (e - t0):7.2f} ms  {k:4d} kernels  busy {b / 1e6:6.2f}  '
                  f'{short(a)[:38]:38s} .. {short(z)[:38]}')
        tot = {}
        for s0, e0, _, n in seq:
            k = short(n)
            c, t = tot.get(k, (0, 0))
            tot[k] = (c + 1, t + e0 - s0)
        print(f'  top kernels on stream {q} this step:')
        for k, (c, t) in sorted(tot.items(), key=lambda kv: -kv[1][1])[:25]:
            print(f'    {t / 1e3:9.1f} us  {c:4d}x  {k[:90]}')


if __name__ == '__main__':
    main()
