set -o pipefail
for g in "64,192,64,34" "32,96,64,34" "16,48,32,34" "16,48,16,16" "32,64,32,34" "8,32,16,16"; do
  echo "grid=$g $(BPE_SPEC_GRID=$g timeout -k 10 60 python tools/c1_prof.py | python3 -c 'import json,sys; d=json.load(sys.stdin); s=d["stats"]; print(d["ms"], s["merges"])')" || exit 1
done
