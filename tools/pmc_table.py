"""Average each PMC counter over the dispatches of the dominant kernel in tools/pmc_gemm.sh output.
usage: python tools/pmc_table.py gpurun_out/pmc_g/ff1 [kernel-substring]"""
import csv
import glob
import os
import sys
from collections import defaultdict


def main():
    root = sys.argv[1]
    sub = sys.argv[2] if len(sys.argv) > 2 else 'gemm256_kernel'
    vals = defaultdict(list)
    durs = []
    for f in sorted(glob.glob(os.path.join(root, 'p*', '**', '*counter_collection.csv'), recursive=True)):
        for r in csv.DictReader(open(f)):
            if sub in r['Kernel_Name']:
                vals[r['Counter_Name']].append(float(r['Counter_Value']))
                durs.append((int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1e3)
    for k, v in sorted(vals.items()):
        print(f'{k:32s} {sum(v) / len(v):16.1f}   (n={len(v)})')
    print(f'{"duration_us (profiled)":32s} {sum(durs) / len(durs):16.1f}')


if __name__ == '__main__':
    main()
