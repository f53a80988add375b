set -u
O=gpurun_out/r05_pcmap; mkdir -p $O
for cfg in "ECG_GRID_MAP=3" "ECG_GRID_MAP=1" "ECG_GRID_MAP=2 ECG_MAP_GROUP=4" "ECG_GRID_MAP=2 ECG_MAP_GROUP=16" "ECG_GRID_MAP=0" "ECG_GRID_MAP=3"; do
  env $cfg timeout -k 10 200 python bench.py --workload pc-merge --forms rows,fused --steps 10 --warmup 2 --no-cpu-baseline > $O/tmp.log 2>&1 || exit 1
  echo "$cfg | $(tail -1 $O/tmp.log | python -c 'import json,sys; d=json.loads(sys.stdin.read())["results"]; print({k: v["algorithmic_frac"] for k, v in d.items()})')" | tee -a $O/pcmap.txt
done
