"""Per-basic-block instruction mix of the hottest (most-MFMA) blocks of each kernel in a
hipcc -S device assembly file: MFMA / VALU / SALU / LDS / VMEM counts, to check a main loop's
VALU-per-MFMA budget without a GPU.

    python scripts/tools/asm_loops.py kernel.s [name-filter] [top-blocks]
"""
import re
import sys
from collections import Counter


def classify(op):
    if 'mfma' in op:
        return 'mfma'
    if op.startswith('ds_read') or op.startswith('ds_load'):
        return 'ds_rd'
    if op.startswith('ds_write') or op.startswith('ds_store'):
        return 'ds_wr'
    if op.startswith('buffer_load') or op.startswith('global_load'):
        return 'vmem_ld'
    if op.startswith('buffer_store') or op.startswith('global_store'):
        return 'vmem_st'
    if op.startswith('v_'):
        return 'valu'
    if op.startswith('s_waitcnt') or op.startswith('s_barrier'):
        return 'sync'
    if op.startswith('s_'):
        return 'salu'
    return 'other'


def main():
    path = sys.argv[1]
    filt = sys.argv[2] if len(sys.argv) > 2 else ''
    top = int(sys.argv[3]) if len(sys.argv) > 3 else 2
    fn = None
    blocks = {}
    cur = None
    for line in open(path):
        s = line.strip()
        m = re.match(r'^(_Z\S+):\s*(;.*)?$', s)
        if m:
            fn = m.group(1)
            cur = (fn, 'entry')
            blocks[cur] = Counter()
            continue
        if fn is None:
            continue
        m = re.match(r'^(\.LBB\S+):', s)
        if m:
            cur = (fn, m.group(1))
            blocks[cur] = Counter()
            continue
        if not s or s.startswith(';') or s.startswith('.') or s.endswith(':'):
            continue
        op = s.split()[0]
        blocks[cur][classify(op)] += 1
    byfn = {}
    for (f, b), c in blocks.items():
        if filt and filt not in f:
            continue
        byfn.setdefault(f, []).append((c['mfma'], b, c))
    for f, lst in sorted(byfn.items()):
        lst.sort(reverse=True, key=lambda t: t[0])
        if not lst or lst[0][0] == 0:
            continue
        print(f[:110])
        for n, b, c in lst[:top]:
            if n == 0:
                break
            print('   %-10s mfma %4d valu %4d (%.2f/mfma) salu %3d ds_rd %3d ds_wr %3d vmem %3d sync %3d' % (
                b, n, c['valu'], c['valu'] / n, c['salu'], c['ds_rd'], c['ds_wr'], c['vmem_ld'],
                c['sync']))


if __name__ == '__main__':
    main()
