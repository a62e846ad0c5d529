"""Share of a pipelined kernel trace (rocprofv3 --kernel-trace CSV) by the set of stage classes running:
'fd' = FAST or describe running; otherwise the combination of latency-bound stages (quadtree, pyramid,
SearchForInitialization) or idle.  Window: [lo, hi] ms from the first kernel (default: 80 ms to 20 ms before
the last kernel, the timed region of bench.py's default run under rocprofv3)."""
import csv, sys
path = sys.argv[1]
rows = list(csv.DictReader(open(path)))
t0 = min(int(r['Start_Timestamp']) for r in rows)
t1 = max(int(r['End_Timestamp']) for r in rows)
lo = t0 + float(sys.argv[2]) * 1e6 if len(sys.argv) > 2 else t0 + 80e6
hi = t0 + float(sys.argv[3]) * 1e6 if len(sys.argv) > 3 else t1 - 20e6
ev = []
for r in rows:
    n = r['Kernel_Name'].split('(')[0]
    c = 'fd' if ('fast' in n or 'describe' in n) else 'qt' if 'quadtree' in n else 'pyr' if 'pyramid' in n \
        else 'si' if 'si_' in n else 'other'
    ev.append((int(r['Start_Timestamp']), 1, c))
    ev.append((int(r['End_Timestamp']), -1, c))
ev.sort()
act = dict.fromkeys(['fd', 'qt', 'pyr', 'si', 'other'], 0)
acc, prev = {}, None
for t, d, c in ev:
    if prev is not None:
        a, b = max(prev, lo), min(t, hi)
        if b > a:
            k = 'fd' if act['fd'] else ('+'.join(sorted(x for x, v in act.items() if v)) or 'idle')
            acc[k] = acc.get(k, 0) + (b - a)
    act[c] += d
    prev = t
tot = sum(acc.values())
for k, v in sorted(acc.items(), key=lambda x: -x[1]):
    if v / tot >= 0.001:
        print("%-16s %5.1f%%" % (k, 100 * v / tot))
