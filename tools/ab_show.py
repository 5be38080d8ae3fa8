"""Summarise tools/ab_lib.sh outputs: python3 tools/ab_show.py TAG"""
import glob, json, sys
tag = sys.argv[1]
for f in sorted(glob.glob(f"gpurun_out/ab_*_{tag}*.json")):
    try:
        d = json.loads(open(f).read().strip().splitlines()[-1])
    except Exception as e:
        print(f, "unreadable", e)
        continue
    b = d.get("breakdown_ms", {})
    print(f"{f:45s} value {d['value']/1e6:7.3f}M  ms/step {d['ms_per_step']:.4f}  init {b.get('init')}  loop {b.get('loop')}  K {d['roofline']['avg_ms']*1e3:.2f}us")
