"""Summarise a captured hipGraph's DOT dump (``IMAGINAIRE_AMD_GRAPH_DOT=path`` makes
utils/cuda_graph.py write one with hipGraphDebugDotPrint): node kinds, in/out degrees, roots,
and whether the graph is one linear chain — every node's producer has an edge to it.

    python scripts/probe/graph_dot.py graph.dot
"""
import collections
import re
import sys


def parse(path):
    txt = open(path, errors='replace').read()
    edge_re = re.compile(r'"?([\w.]+)"?\s*->\s*"?([\w.]+)"?')
    node_re = re.compile(r'^\s*"?([\w.]+)"?\s*\[(.*)\]\s*;?\s*$')
    nodes, edges = {}, []
    # (labels span lines in some dumps: join bracketed blocks first)
    buf, depth, stmts = '', 0, []
    for ch in txt:
        buf += ch
        if ch == '[':
            depth += 1
        elif ch == ']':
            depth -= 1
        elif ch in ';\n' and depth == 0:
            stmts.append(buf.strip())
            buf = ''
    stmts.append(buf.strip())
    for s in stmts:
        if not s:
            continue
        m = edge_re.search(s)
        if m and '->' in s.split('[')[0]:
            edges.append((m.group(1), m.group(2)))
            continue
        m = node_re.match(s.replace('\n', ' '))
        if m and m.group(1) not in ('graph', 'node', 'edge', 'digraph', 'subgraph'):
            nodes[m.group(1)] = m.group(2)
    return nodes, edges


def kind(label):
    u = label.upper()
    for k in ('MEMCPY', 'MEMSET', 'EVENT_RECORD', 'EVENT_WAIT', 'EVENTRECORD', 'WAITEVENT',
              'HOST', 'EMPTY', 'CHILD', 'KERNEL'):
        if k in u:
            return k
    return 'OTHER'


def main():
    nodes, edges = parse(sys.argv[1])
    indeg, outdeg = collections.Counter(), collections.Counter()
    for a, b in edges:
        outdeg[a] += 1
        indeg[b] += 1
    kinds = collections.Counter(kind(l) for l in nodes.values())
    print('nodes %d, edges %d' % (len(nodes), len(edges)))
    print('node kinds:', dict(kinds))
    roots = [n for n in nodes if indeg[n] == 0]
    print('roots (in-degree 0): %d' % len(roots), roots[:5])
    print('in-degree histogram:', dict(collections.Counter(indeg[n] for n in nodes)))
    print('out-degree histogram:', dict(collections.Counter(outdeg[n] for n in nodes)))
    chain = len(roots) == 1 and all(indeg[n] <= 1 and outdeg[n] <= 1 for n in nodes)
    print('linear chain:', chain)
    shown = collections.Counter()
    for n, l in nodes.items():
        k = kind(l)
        if shown[k] < 2:
            shown[k] += 1
            print('  example %-8s %s: %s' % (k, n, re.sub(r'\s+', ' ', l)[:300]))
    # non-kernel nodes and their neighbourhood
    succ = collections.defaultdict(list)
    pred = collections.defaultdict(list)
    for a, b in edges:
        succ[a].append(b)
        pred[b].append(a)
    def kname(n):
        m = re.search(r'KERNEL \| \{ID \| \d+ \| ([^\\<]+)', nodes.get(n, ''))
        return m.group(1)[:90] if m else kind(nodes.get(n, ''))

    odd = [n for n, l in nodes.items() if kind(l) not in ('KERNEL',)]
    print('non-kernel nodes: %d' % len(odd))
    pairs = collections.Counter()
    for n in odd:
        pairs[(kind(nodes[n]), tuple(kname(p) for p in pred[n]), tuple(kname(q) for q in succ[n]))] += 1
    print('non-kernel node neighbourhoods (kind, predecessor kernel, successor kernel): count')
    for (k, pr, sc), c in pairs.most_common(40):
        print('  %4d  %-7s %s -> %s' % (c, k, pr, sc))
    for n in [n for n in odd if kind(nodes[n]) == 'MEMSET'][:6]:
        print('  memset %s: %s' % (n, re.sub(r'\s+', ' ', nodes[n])[:400]))


if __name__ == '__main__':
    main()
