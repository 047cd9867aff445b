"""Per-launch summary of tools/pmc_gemm.sh passes for the dominant kernel (most dispatches with the
largest grid): HBM-side traffic and MFMA utilisation, with the gfx950 corrections of
MI355X_MICROARCH.md §HBM / §rocprofv3 (FETCH_SIZE and WRITE_SIZE in KiB, FETCH_SIZE x2 for 16-B
streaming reads; GRBM_GUI_ACTIVE summed over the 8 XCDs; SQ_VALU_MFMA_BUSY_CYCLES summed over
the 1,024 SIMDs).   usage: python tools/pmc_gemm_json.py <pass-dir> <kernel-substring>"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict


def main():
    root, sub = sys.argv[1], sys.argv[2]
    vals = defaultdict(list)
    durs = []
    names = set()
    for f in sorted(glob.glob(os.path.join(root, 'p*', '**', '*counter_collection.csv'), recursive=True)):
        for r in csv.DictReader(open(f)):
            if sub in r['Kernel_Name']:
                names.add(r['Kernel_Name'])
                vals[r['Counter_Name']].append(float(r['Counter_Value']))
                durs.append((int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1e3)
    avg = {k: sum(v) / len(v) for k, v in vals.items()}
    res = {'kernel': sorted(names), 'dispatches': {k: len(v) for k, v in vals.items()},
           'duration_us_profiled': sum(durs) / max(1, len(durs)), 'counters': avg}
    if 'FETCH_SIZE' in avg:
        res['fetch_bytes_per_launch'] = 2.0 * 1024.0 * avg['FETCH_SIZE']
    if 'WRITE_SIZE' in avg:
        res['write_bytes_per_launch'] = 1024.0 * avg['WRITE_SIZE']
    if 'FETCH_SIZE' in avg and 'WRITE_SIZE' in avg:
        res['traffic_bytes_per_launch'] = res['fetch_bytes_per_launch'] + res['write_bytes_per_launch']
    if 'SQ_VALU_MFMA_BUSY_CYCLES' in avg and 'GRBM_GUI_ACTIVE' in avg:
        xcd_cycles = avg['GRBM_GUI_ACTIVE'] / 8.0
        res['mfma_busy'] = avg['SQ_VALU_MFMA_BUSY_CYCLES'] / (xcd_cycles * 1024.0)
        res['clock_ghz'] = xcd_cycles / (res['duration_us_profiled'] * 1e3) if durs else None
    if 'TCC_HIT_sum' in avg and 'TCC_MISS_sum' in avg:
        res['l2_hit_rate'] = avg['TCC_HIT_sum'] / max(1.0, avg['TCC_HIT_sum'] + avg['TCC_MISS_sum'])
    res['method'] = ('rocprofv3 --pmc, one counter group per pass (tools/pmc_gemm.sh); FETCH_SIZE x2 x 1024, '
                     'WRITE_SIZE x 1024; mfma_busy = SQ_VALU_MFMA_BUSY_CYCLES / (GRBM_GUI_ACTIVE / 8 x 1024 SIMDs)')
    print(json.dumps(res, indent=1))


if __name__ == '__main__':
    main()
