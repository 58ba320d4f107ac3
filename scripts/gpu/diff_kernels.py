"""Per-kernel difference of two summarize_kernels.py outputs (B - A), largest first.

    python scripts/gpu/diff_kernels.py kernels_plain.txt kernels_forced.txt [rows]
"""
import re
import sys


def load(path):
    out, wall = {}, None
    for line in open(path):
        m = re.match(r'STEADY STATE .*wall span ([\d.]+) ms', line)
        if m:
            wall = float(m.group(1))
        m = re.match(r'\s+([\d.]+) ms\s+[\d.]+%\s+(\d+)\s+(.*)', line)
        if m:
            name = m.group(3).strip()[:110]
            t, n = out.get(name, (0.0, 0))
            out[name] = (t + float(m.group(1)), n + int(m.group(2)))
    return out, wall


def main():
    a, wa = load(sys.argv[1])
    b, wb = load(sys.argv[2])
    rows = int(sys.argv[3]) if len(sys.argv) > 3 else 25
    print('wall span: %s -> %s ms' % (wa, wb))
    diff = []
    for k in set(a) | set(b):
        ta, na = a.get(k, (0.0, 0))
        tb, nb = b.get(k, (0.0, 0))
        diff.append((tb - ta, nb - na, k))
    diff.sort(key=lambda r: -abs(r[0]))
    for d, dn, k in diff[:rows]:
        print('%+8.2f ms %+6d calls  %s' % (d, dn, k))


if __name__ == '__main__':
    main()
