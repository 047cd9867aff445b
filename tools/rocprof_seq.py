"""Every kernel of one contrastive step on one stream, in launch order, with its offset from the
step's first main-stream kernel and its duration (rocprofv3 kernel trace, rocpd sqlite) -- to place
a kernel of the summary in the step.
usage: python tools/rocprof_seq.py <results.db> [stream_id] [step_marker_substring]"""
import sqlite3
import sys


def main():
    db = sqlite3.connect(sys.argv[1])
    arg = sys.argv[2] if len(sys.argv) > 2 else None
    every = arg == 'all'
    sid = int(arg) if arg not in (None, 'all') else None
    marker = sys.argv[3] if len(sys.argv) > 3 else 'patch_ln_strip'
    rows = sorted(db.execute('select start, "end", stream_id, name from kernels').fetchall())
    starts = [r[0] for r in rows if marker in r[3]]
    if len(starts) < 3:
        print('fewer than 3 step markers'); return
    # the last interval between markers that is a whole train step: bench.py's forward-only
    # measurements (vit_forward / vit_forward_eval) come after the steps and are much shorter
    # (and the first, warm-up steps are much longer: the last step-sized interval, by the median)
    gaps = [(b - a, a, b) for a, b in zip(starts, starts[1:])]
    med = sorted(g[0] for g in gaps)[len(gaps) // 2]
    t0, t1 = [(a, b) for g, a, b in gaps if 0.7 * med <= g <= 1.5 * med][-1]
    if sid is None:
        sid = next(r[2] for r in rows if r[0] == t0)
    print(f'step {1e-6 * (t1 - t0):.2f} ms, stream {"all" if every else sid}')
    for s, e, q, n in rows:
        if t0 <= s < t1 and (every or q == sid):
            n = n.replace('(anonymous namespace)::', '').replace('void ', '').split('(')[0]
            tag = f'[{q}] ' if every else ''
            print(f'{1e-6 * (s - t0):8.3f} ms  {1e-3 * (e - s):8.1f} us  {tag}{n[:100]}')


if __name__ == '__main__':
    main()
