set -u
O=gpurun_out/r05_sweep; mkdir -p $O
for cfg in "ECG_GRID_MAP=1" "ECG_GRID_MAP=2 ECG_MAP_GROUP=1" "ECG_GRID_MAP=2 ECG_MAP_GROUP=4" "ECG_GRID_MAP=2 ECG_MAP_GROUP=64" "ECG_GRID_MAP=1 ECG_COLS_PER_WG=256" "ECG_GRID_MAP=1 ECG_COLS_PER_WG=512" "ECG_GRID_MAP=1 ECG_NT=1" "ECG_GRID_MAP=1 ECG_NT=2" "ECG_GRID_MAP=1 ECG_NT=0"; do
  env $cfg timeout -k 10 60 ./tools/movement_ceiling 3 10 4096 enc_general > $O/tmp.txt 2>&1 || exit 1
  echo "$cfg | $(tail -1 $O/tmp.txt)" | tee -a $O/sweep.txt
done
