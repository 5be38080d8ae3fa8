"""print the key fields of bench JSON lines (last line of each file)"""
import json
import sys

for f in sys.argv[1:]:
    try:
        d = json.loads(open(f).read().strip().splitlines()[-1])
    except Exception as e:  # noqa: BLE001
        print(f, "unreadable:", e)
        continue
    eng = d.get("engine", {})
    print(f, d.get("value"), d.get("ms_per_step"), "speedup", d.get("speedup_vs_1gpu"), "same", d.get("identical_to_1gpu"),
          d.get("breakdown_ms"), "batches", eng.get("batches"), d.get("error", ""))
