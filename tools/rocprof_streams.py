"""Per-stream (queue) busy time of a rocprofv3 kernel trace (rocpd sqlite): how much of the wall
time each queue keeps the GPU busy, and the union over queues, for the last `window_ms`.
usage: python tools/rocprof_streams.py <results.db> [window_ms]"""
import sqlite3
import sys


def union_len(iv):
    tot, cur_s, cur_e = 0, None, None
    for s, e in sorted(iv):
        if cur_e is None or s > cur_e:
            if cur_e is not None:
                tot += cur_e - cur_s
            cur_s, cur_e = s, e
        else:
            cur_e = max(cur_e, e)
    if cur_e is not None:
        tot += cur_e - cur_s
    return tot


def main():
    db = sqlite3.connect(sys.argv[1])
    window = float(sys.argv[2]) if len(sys.argv) > 2 else 200.0
    cols = [r[1] for r in db.execute("pragma table_info('kernels')")]
    qcol = next((c for c in ('stream_id', 'queue_id', 'queue') if c in cols), None)
    print('columns:', ', '.join(cols))
    rows = db.execute(f'select start, "end", {qcol}, name from kernels').fetchall()
    t1 = max(r[1] for r in rows)
    t0 = t1 - window * 1e6
    rows = [r for r in rows if r[0] >= t0]
    by_q = {}
    for s, e, q, n in rows:
        by_q.setdefault(q, []).append((s, e))
    print(f'window {window:.1f} ms, {len(rows)} kernels, queue column {qcol}')
    for q, iv in sorted(by_q.items(), key=lambda kv: -len(kv[1])):
        print(f'  {qcol} {q}: {len(iv):6d} kernels, busy {union_len(iv) / 1e6:8.2f} ms')
    print(f'  union busy {union_len([(s, e) for s, e, _, _ in rows]) / 1e6:8.2f} ms of {window:.1f}')
    # largest idle gaps of the busiest queue, with the kernels on either side
    q0 = max(by_q, key=lambda q: union_len(by_q[q]))
    seq = sorted((s, e, n) for s, e, q, n in rows if q == q0)
    gaps = []
    end = seq[0][1]
    for i in range(1, len(seq)):
        if seq[i][0] > end:
            gaps.append((seq[i][0] - end, seq[i - 1][2], seq[i][2]))
        end = max(end, seq[i][1])
    gaps.sort(reverse=True)
    tot = sum(g for g, _, _ in gaps)
    print(f'  {qcol} {q0}: {len(gaps)} gaps, {tot / 1e6:.2f} ms idle; largest:')
    for g, a, b in gaps[:25]:
        print(f'    {g / 1e3:8.1f} us  after {a[:60]:60s} before {b[:60]}')


if __name__ == '__main__':
    main()
