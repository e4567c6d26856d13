set -e
for dt in f32 f64; do for tb in ${TBS:-4194304 8388608 16777216 33554432}; do
  echo "== DT=$dt tile_bytes=$tb"
  DT=$dt GRF_SPMM_TILE_BYTES=$tb timeout -k 10 200 python tools/cg_time.py 2>&1 | grep -E "^cg max_iter=50|pathwise"
done; done
