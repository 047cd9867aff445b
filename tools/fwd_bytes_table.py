"""Summarise tools/fwd_bytes.sh: the LAST train step's 3D-ViT forward (from the last patch LayerNorm
to the VQ select), per dispatch in order and per kernel kind, FETCH_SIZE x 2 (gfx950 reports half
the bytes of 16-B/lane streaming reads; L2 misses, MALL hits included: an upper bound on HBM reads)
and WRITE_SIZE, in MB (1e6 B).   usage: python tools/fwd_bytes_table.py <pmc dir>"""
import csv
import glob
import os
import sys
from collections import OrderedDict


def load(d, counter):
    rows = []
    for f in glob.glob(os.path.join(d, counter, '**', '*counter_collection.csv'), recursive=True):
        for r in csv.DictReader(open(f)):
            if r['Counter_Name'] == counter:
                rows.append((int(r['Start_Timestamp']), r['Kernel_Name'], float(r['Counter_Value'])))
    rows.sort()
    return rows


def window(rows):
    starts = [i for i, r in enumerate(rows) if 'patch_ln' in r[1]]
    i0 = starts[-1]
    i1 = next(i for i in range(i0, len(rows)) if 'vq_select' in rows[i][1])
    return rows[i0:i1 + 1]


def short(n):
    n = n.replace('(anonymous namespace)::', '').replace('void ', '')
    return n.split('(')[0][:70]


def main():
    d = sys.argv[1]
    f, w = window(load(d, 'FETCH_SIZE')), window(load(d, 'WRITE_SIZE'))
    # the two passes run the same program: pair the window's dispatches by kernel-name order
    assert [short(r[1]) for r in f] == [short(r[1]) for r in w], 'passes differ'
    KiB = 1024 / 1e6
    print(f'{"#":>3s} {"kernel":70s} {"read MB":>9s} {"write MB":>9s}')
    agg = OrderedDict()
    tr = tw = 0.0
    for i, (a, b) in enumerate(zip(f, w)):
        rd, wr = 2 * a[2] * KiB, b[2] * KiB
        tr += rd
        tw += wr
        k = short(a[1])
        print(f'{i:3d} {k:70s} {rd:9.1f} {wr:9.1f}')
        s = agg.setdefault(k, [0, 0.0, 0.0])
        s[0] += 1
        s[1] += rd
        s[2] += wr
    print(f'\nper kernel kind (whole forward, {len(f)} dispatches): read {tr / 1e3:.2f} GB, write {tw / 1e3:.2f} GB')
    for k, (n, rd, wr) in sorted(agg.items(), key=lambda kv: -(kv[1][1] + kv[1][2])):
        print(f'{n:3d} x {k:70s} {rd:9.1f} {wr:9.1f}')


if __name__ == '__main__':
    main()
