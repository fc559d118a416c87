import csv, json, sys
rows = list(csv.DictReader(open('gpurun_out/prof/run_kernel_stats.csv')))
for r in rows[:14]:
    print(f"{r['Name'][:60]:60s} calls={r['Calls']:>5} avg_ms={float(r['AverageNs'])/1e6:8.3f} pct={float(r['Percentage']):.1f}")
b = [l for l in open('gpurun_out/bench.log') if l.startswith('{')]
if b:
    j = json.loads(b[-1])
    print(f"{j['value']/1e9:.3f} Gev/s  {j['ms_per_step']:.2f} ms/step  phases={j['phase_ms']}  frac={j['roofline']['frac']:.4f}  verified={j['verified_vs_restatement']}")
