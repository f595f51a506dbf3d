set -u
O=gpurun_out/qab; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_quic.py -x -q -m gpu --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || exit 1
for v in default qw3 qw2; do
  if [ $v = default ]; then L=hysteria_amd/libhyobfs.so; else L=build_variants/libhyobfs_$v.so; fi
  HYOBFS_LIB=$L timeout -k 10 200 python -u scripts/bench_quic.py > $O/bench_$v.json 2>&1 || exit 1
done
echo done
