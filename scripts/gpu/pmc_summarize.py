"""Summarise rocprofv3 --pmc counter CSVs (gpurun_out/pmc/<mode>_<pass>.csv) per kernel:
mean counter value per dispatch, plus derived VALU:MFMA and wait ratios."""
import collections
import csv
import glob
import os
import sys


def main(root):
    per = collections.defaultdict(lambda: collections.defaultdict(list))
    for f in sorted(glob.glob(os.path.join(root, '*_*.csv'))):
        mode = os.path.basename(f).split('_')[0]
        with open(f) as fh:
            for row in csv.DictReader(fh):
                name = row.get('Kernel_Name', row.get('Kernel-Name', '?'))
                if 'conv' not in name and 'wgrad' not in name:
                    continue
                ctr = row.get('Counter_Name', row.get('Counter-Name'))
                val = float(row.get('Counter_Value', row.get('Counter-Value', 0)))
                per[(mode, name.split('(')[0][-60:])][ctr].append(val)
    for (mode, name), ctrs in sorted(per.items()):
        shp = os.path.join(root, mode + '.shape')
        extra = open(shp).read().strip() if os.path.exists(shp) else ''
        print('== %s  %s  %s' % (mode, extra, name))
        mean = {c: sum(v) / len(v) for c, v in ctrs.items()}
        for c in sorted(mean):
            print('  %-24s %16.0f' % (c, mean[c]))
        if mean.get('SQ_INSTS_MFMA'):
            print('  VALU:MFMA instr ratio    %16.2f' % (mean.get('SQ_INSTS_VALU', 0) /
                                                      mean['SQ_INSTS_MFMA']))
        if mean.get('SQ_VALU_MFMA_BUSY_CYCLES') and mean.get('GRBM_GUI_ACTIVE'):
            # MFMA busy cycles summed over 1024 SIMDs vs the kernel's GPU-active cycles (summed
            # over 8 XCDs by rocprofv3): fraction of SIMD-cycles the matrix pipe was busy
            print('  MFMA busy fraction       %16.3f' % (
                mean['SQ_VALU_MFMA_BUSY_CYCLES'] / (mean['GRBM_GUI_ACTIVE'] / 8 * 1024)))
        if mean.get('TCC_HIT_sum') is not None and mean.get('TCC_MISS_sum') is not None:
            h, m = mean['TCC_HIT_sum'], mean['TCC_MISS_sum']
            print('  L2 hit rate              %16.3f' % (h / max(h + m, 1)))
        if mean.get('SQ_BUSY_CYCLES') and mean.get('SQ_ACTIVE_INST_MFMA'):
            print('  MFMA-active / busy       %16.2f' % (mean['SQ_ACTIVE_INST_MFMA'] /
                                                      mean['SQ_BUSY_CYCLES']))


if __name__ == '__main__':
    main(sys.argv[1] if len(sys.argv) > 1 else 'gpurun_out/pmc')
