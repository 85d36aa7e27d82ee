#!/bin/bash
# configs[4]'s structure on ONE GPU, outside torchrun (no sleeping torch contexts): 5
# ranks = 4 + idle spare, Raben 256 MiB float32 SUM, six calls per job; no fault, and a
# kill mid-exchange in call 2 in reduce-scatter step 1 and in the last allgather step
# (both recover).  Per call: max-over-ranks ms, recoveries, comm size, exact-sum check.
#   bash tools/c5_one_gpu.sh [OUT]          (OUT defaults to gpurun_out/c5_one_gpu)
set -u
OUT=${1:-gpurun_out/c5_one_gpu}
mkdir -p "$OUT"
B=fault-tolerant_amd/bin
for k in none 4:1:1:3:2 4:2:0:3:2; do
  if [ "$k" = none ]; then unset FTAR_KILL; else export FTAR_KILL=$k; fi
  tag=${k//:/_}
  timeout -k 10 120 $B/ftrun -np 5 --devmap 0,0,0,0,0 $B/ftbench raben 67108864 6 > "$OUT/$tag.json" 2> "$OUT/$tag.err"
  rc=$?
  echo "kill $k rc=$rc"
  [ $rc -ne 0 ] && { tail -5 "$OUT/$tag.err"; exit $rc; }
done
python3 - "$OUT" <<'PY'
import json, os, sys
out = sys.argv[1]
res = {}
for tag in ("none", "4_1_1_3_2", "4_2_0_3_2"):
    ranks = [json.loads(l) for l in open(os.path.join(out, tag + ".json")) if l.startswith("{")]
    calls = []
    for c in range(6):
        per = [r["calls"][c] for r in ranks]
        calls.append({"ms": round(max(p["ms"] for p in per), 3), "recoveries": max(p["recoveries"] for p in per),
                      "comm_size": min(p["comm_size"] for p in per), "value": per[0]["value"],
                      "uniform": all(p["uniform"] and p["value"] == per[0]["value"] for p in per)})
    res[tag] = {"survivors": len(ranks), "calls": calls}
json.dump(res, open(os.path.join(out, "summary.json"), "w"), indent=1)
print(json.dumps(res))
PY
