timeout -k 5 120 python -u -m pytest -q -x tests/test_gpu_table_hash.py 2>&1 | tail -3
for hot in 0.5 0.03; do
  echo "== new $hot"; HOT=$hot DQ_FREQ_PATH=atomic timeout -k 5 120 python -u tools/dbg_hot.py 2>&1 | grep -v "^\[W\|amdgpu.ids" | tail -2
done
