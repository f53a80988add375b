# Round 5: encode / decode launch knobs on the product kernel's own path (tools/movement_ceiling).
set -u
O=gpurun_out/r05_sweep2; mkdir -p $O
timeout -k 10 200 ./tools/movement_ceiling 6 10 4096 enc_general maps > $O/maps_encode.txt 2>&1 || exit 1
cat $O/maps_encode.txt
timeout -k 10 200 ./tools/movement_ceiling 6 10 4096 dec_general maps > $O/maps_decode.txt 2>&1 || exit 1
cat $O/maps_decode.txt
