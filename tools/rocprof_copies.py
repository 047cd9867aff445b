"""Account for the runtime's blit kernels (`__amd_rocclr_copyBuffer` / `fillBuffer`: hipMemcpyAsync /
hipMemsetAsync device-side) in a rocprofv3 kernel trace (rocpd sqlite): per stream, how many per
step, their time, whether the stream's next kernel had to wait for them (a copy ends less than 2 us
before the next kernel on its stream starts = on that stream's path), and the kernels around them
(which op issued them).
usage: python tools/rocprof_copies.py <results.db> [steps] [window_ms]"""
import collections
import sqlite3
import sys


def short(n):
    n = n.replace('(anonymous namespace)::', '').replace('void ', '')
    return n.split('(')[0][:58]


def main():
    db = sqlite3.connect(sys.argv[1])
    steps = float(sys.argv[2]) if len(sys.argv) > 2 else 1.0
    window = float(sys.argv[3]) if len(sys.argv) > 3 else 0.0
    cols = [r[1] for r in db.execute("pragma table_info('kernels')")]
    qcol = next((c for c in ('stream_id', 'queue_id', 'queue') if c in cols), None)
    gx = 'grid_x' if 'grid_x' in cols else None
    rows = db.execute(f'select start, "end", {qcol}, name{", " + gx if gx else ""} from kernels').fetchall()
    if window > 0:
        t1 = max(r[1] for r in rows)
        rows = [r for r in rows if r[0] >= t1 - window * 1e6]
    by_q = collections.defaultdict(list)
    for r in rows:
        by_q[r[2]].append(r)
    for q in by_q:
        by_q[q].sort()
    print(f'{qcol}: blit kernels per stream ({steps:g} steps)')
    for q, seq in sorted(by_q.items()):
        blits = [i for i, r in enumerate(seq) if '__amd_rocclr' in r[3]]
        if not blits:
            continue
        tot = sum(seq[i][1] - seq[i][0] for i in blits)
        onpath = 0
        ctx = collections.Counter()
        for i in blits:
            nxt = seq[i + 1] if i + 1 < len(seq) else None
            if nxt is not None and nxt[0] - seq[i][1] < 2000:
                onpath += 1
            prev = next((seq[j][3] for j in range(i - 1, -1, -1) if '__amd_rocclr' not in seq[j][3]), '-')
            nx = next((seq[j][3] for j in range(i + 1, len(seq)) if '__amd_rocclr' not in seq[j][3]), '-')
            ctx[(short(seq[i][3]), short(prev), short(nx), seq[i][4] if gx else 0)] += 1
        print(f'  {qcol} {q}: {len(blits) / steps:6.1f} per step, {tot / 1e3 / steps:8.1f} us per step, '
              f'{onpath / steps:5.1f} per step followed within 2 us by the stream\'s next kernel')
        for (n, a, b, g), c in ctx.most_common(30):
            print(f'      {c / steps:5.1f}/step  {n:24s} grid {g:>9}  after {a:58s} before {b}')


if __name__ == '__main__':
    main()
