set -u
bash scripts/gpu_session.sh r04k "test:contig or packed or bimodal or scan or ragged" || exit 1
AB_ARGS="tile" AB_NAME=uniform_saltt AB_LIBS='main=hysteria_amd/libhyobfs.so,saltt=build_variants/libhyobfs_saltt.so' bash scripts/gpu_session.sh r04k ab || exit 1
AB_WORKLOAD=bimodal AB_ARGS="auto,auto@off" AB_NAME=bimodal_scan bash scripts/gpu_session.sh r04k ab || exit 1
R=$GRAFT_REPO_ROOT
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/r04k/trace_bimodal -o run -- python3 $R/scripts/prof_one.py bimodal 10 > $R/gpurun_out/r04k/trace_bimodal.log 2>&1) || exit 1
AB_WORKLOAD=bimodal AB_ARGS="auto@off" AB_NAME=wave_occupancy AB_LIBS='main=hysteria_amd/libhyobfs.so,occ6=build_variants/libhyobfs_occ6.so,occ5=build_variants/libhyobfs_occ5.so,occ4=build_variants/libhyobfs_occ4.so' bash scripts/gpu_session.sh r04k ab || exit 1
AB_NAME=gecko bash scripts/gpu_session.sh r04k test:gecko abg || exit 1
