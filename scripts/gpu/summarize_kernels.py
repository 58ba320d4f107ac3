"""Summarise rocprofv3 --stats kernel tables: top kernels by total time,
grouped into families (MIOpen conv, GEMM, imaginaire_amd HIP kernels, ...)."""
import csv
import glob
import os
import re
import sys


def family(name):
    n = name.lower()
    if 'conv_fwd_mfma' in n:
        return 'imaginaire_amd MFMA conv (k10)'
    if 'iamd' in n or 'imaginaire' in n or any(k in n for k in (
            'stats_partial', 'stats_finalize', 'apply_fwd', 'bwd_reduce', 'bwd_apply',
            'sum_partials', 'bias_act', 'adam_kernel', 'sn_sigma', 'ema_kernel',
            'renorm_kernel', 'mask_window', 'warp_', 'resample2d', 'corr_', 'chnorm')):
        return 'imaginaire_amd HIP'
    if any(k in n for k in ('igemm', 'conv', 'miopen', 'xdlops', 'naive_conv', 'winograd',
                            'sp3asm', 'gridwise')):
        return 'MIOpen conv'
    if any(k in n for k in ('gemm', 'cijk', 'hipblaslt', 'tensile')):
        return 'GEMM (hipBLASLt/rocBLAS)'
    if 'elementwise' in n or 'vectorized' in n or 'unrolled' in n:
        return 'torch elementwise'
    if 'reduce' in n:
        return 'torch reduce'
    if 'cat' in n or 'copy' in n or 'transpose' in n or 'batch_norm' in n:
        return 'torch copy/cat/layout'
    return 'other'


MARKER = 'iamd_profile_marker_kernel'


def steady_rows(root):
    """Per-kernel totals from the kernel trace, counting only dispatches that
    start after the last profile marker (= the timed steady-state region)."""
    traces = glob.glob(os.path.join(root, '**', '*kernel_trace*.csv'), recursive=True)
    if not traces:
        return None, 0.0
    recs = []
    for f in traces:
        with open(f) as fh:
            rd = csv.DictReader(fh)
            kn = next(k for k in rd.fieldnames if 'Kernel_Name' in k)
            ks = next(k for k in rd.fieldnames if 'Start_Timestamp' in k)
            ke = next(k for k in rd.fieldnames if 'End_Timestamp' in k)
            for r in rd:
                recs.append((int(r[ks]), int(r[ke]), r[kn]))
    marks = [s for s, _, n in recs if MARKER in n]
    if not marks:
        return None, 0.0
    t0 = max(marks)
    agg = {}
    t_end = t0
    for s, e, n in recs:
        if s >= t0 and MARKER not in n:
            a = agg.setdefault(n, [0, 0.0])
            a[0] += 1
            a[1] += e - s
            t_end = max(t_end, e)
    rows = [{'Name': n, 'Calls': str(c), 'TotalDurationNs': str(d)} for n, (c, d) in agg.items()]
    return rows, (t_end - t0) / 1e6


def main(root):
    rows, span_ms = steady_rows(root)
    if rows:
        print('STEADY STATE (after last profile marker): wall span %.1f ms' % span_ms)
    else:
        files = glob.glob(os.path.join(root, '**', '*kernel_stats*.csv'), recursive=True)
        rows = []
        for f in files:
            with open(f) as fh:
                for r in csv.DictReader(fh):
                    rows.append(r)
        print('WHOLE RUN (no marker found)')
    if not rows:
        print('no kernel stats found under', root)
        return
    key_name = 'Name' if 'Name' in rows[0] else list(rows[0].keys())[0]
    key_total = next(k for k in rows[0] if 'TotalDuration' in k or k == 'TotalDurationNs')
    key_calls = next((k for k in rows[0] if k.lower() == 'calls'), None)
    total = sum(float(r[key_total]) for r in rows)
    fam = {}
    for r in rows:
        fam.setdefault(family(r[key_name]), 0.0)
        fam[family(r[key_name])] += float(r[key_total])
    print('total kernel time: %.1f ms' % (total / 1e6))
    for k, v in sorted(fam.items(), key=lambda kv: -kv[1]):
        print('  %-28s %9.1f ms  %5.1f%%' % (k, v / 1e6, 100 * v / total))
    print()
    rows.sort(key=lambda r: -float(r[key_total]))
    for r in rows[:int(os.environ.get("SUMMARY_ROWS", "150"))]:
        name = re.sub(r'\s+', ' ', r[key_name])[:110]
        calls = r[key_calls] if key_calls else '?'
        print('%9.2f ms %5.1f%% %6s  %s' % (float(r[key_total]) / 1e6,
                                            100 * float(r[key_total]) / total, calls, name))


if __name__ == '__main__':
    main(sys.argv[1] if len(sys.argv) > 1 else 'gpurun_out/prof')
