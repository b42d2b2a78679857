"""Summary of a C5 kernel timeline (scripts/r06_c5trace.sh output): per-step span, the main stream's kernel time and
launch gaps over the last 10 steps, and the side stream's kernels.  Usage: python scripts/c5_gaps.py DIR"""
import csv, sys, glob, collections
f = glob.glob(sys.argv[1] + '/**/*kernel_trace.csv', recursive=True)[0]
rows = list(csv.DictReader(open(f)))
print(rows[0].keys())
key = 'Stream_Id' if 'Stream_Id' in rows[0] else 'Queue_Id'
by = collections.defaultdict(list)
for r in rows:
    by[r[key]].append((int(r['Start_Timestamp']), int(r['End_Timestamp']), r['Kernel_Name'][:60]))
for q, ks in by.items():
    ks.sort()
    print('stream', q, 'kernels', len(ks))
# main stream = the one with the most wq_horner_pc kernels
main = max(by, key=lambda q: sum('horner_pc' in k[2] for k in by[q]))
ks = by[main]
# last 10 steps: find the last 10*12 GEMMs
gem = [k for k in ks if 'horner' in k[2]]
last = gem[-120:]
t0, t1 = last[0][0], last[-1][1]
busy = sum(e - s for s, e, _ in last)
span_ks = [k for k in ks if k[0] >= t0 and k[1] <= t1]
busy_all = sum(e - s for s, e, _ in span_ks)
gaps = [span_ks[i + 1][0] - span_ks[i][1] for i in range(len(span_ks) - 1)]
print('span per step us %.1f' % ((t1 - t0) / 10 / 1e3), 'gemm busy per step %.1f' % (busy / 10 / 1e3),
      'main busy per step %.1f' % (busy_all / 10 / 1e3), 'kernels', len(span_ks))
gaps.sort()
print('gaps us: median %.2f p90 %.2f max %.2f sum/step %.1f' % (gaps[len(gaps)//2]/1e3, gaps[int(len(gaps)*.9)]/1e3, gaps[-1]/1e3, sum(gaps)/10/1e3))
names = collections.Counter(k[2] for k in span_ks)
print(names.most_common(10))
other = [q for q in by if q != main]
for q in other:
    o = [k for k in by[q] if k[0] >= t0 and k[1] <= t1]
    print('side', q, len(o), 'busy per step %.1f' % (sum(e - s for s, e, _ in o) / 10 / 1e3), collections.Counter(k[2] for k in o).most_common(6))
