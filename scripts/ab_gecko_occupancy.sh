# Gecko encode with fewer workgroups per CU (unused dynamic LDS, HYOBFS_GK_LDS_PAD):
# 0 = 5 workgroups/CU (VGPR-limited), 36000 B = 4, 48000 B = 3, 70000 B = 2.
set -u
O=gpurun_out/gk_occ; mkdir -p $O
for i in 1 2; do
  for pad in 0 36000 48000 70000; do
    HYOBFS_GK_LDS_PAD=$pad timeout -k 10 120 python scripts/aux_bench.py > $O/pad${pad}_$i.json 2>$O/err || exit 1
  done
done
echo ok
