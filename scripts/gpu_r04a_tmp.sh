set -u
bash scripts/gpu_session.sh r04a test || exit 1
AB_WORKLOAD=bimodal AB_ARGS="auto,auto@off,wave" AB_NAME=bimodal_layouts bash scripts/gpu_session.sh r04a ab bench trace || exit 1
AB_WORKLOAD=bimodal AB_ARGS="auto" AB_NAME=bimodal_variants AB_LIBS=main=hysteria_amd/libhyobfs.so,s4u4=build_variants/libhyobfs_s4u4.so,s6u2=build_variants/libhyobfs_s6u2.so,t32=build_variants/libhyobfs_t32.so,t8=build_variants/libhyobfs_t8.so bash scripts/gpu_session.sh r04a ab || exit 1
AB_NAME=gecko bash scripts/gpu_session.sh r04a abg aux pmc:main:uniform_deobf:FETCH_SIZE pmc:saltt:uniform_deobf:FETCH_SIZE || exit 1
