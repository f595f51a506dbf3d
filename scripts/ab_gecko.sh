# A/B of Gecko encode variants on one box: GPU Gecko tests, then aux_bench for the
# shipped library and each build_variants/libhyobfs_<name>.so given, alternated.
set -u
O=gpurun_out/gk; mkdir -p $O
timeout -k 10 200 python -u -m pytest tests/test_gpu_gecko.py -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || exit 1
for i in 1 2; do
  timeout -k 10 120 python scripts/aux_bench.py > $O/ship_$i.json 2>$O/err || exit 1
  for v in "$@"; do
    HYOBFS_LIB=$PWD/build_variants/libhyobfs_$v.so timeout -k 10 120 python scripts/aux_bench.py > $O/${v}_$i.json 2>$O/err || exit 1
  done
done
echo ok
