set -u
bash scripts/gpu_session.sh r04j test:contig || exit 1
AB_WORKLOAD=bimodal AB_ARGS="auto,auto@off" AB_NAME=bimodal_prepass AB_LIBS='main=hysteria_amd/libhyobfs.so' bash scripts/gpu_session.sh r04j ab || exit 1
R=$GRAFT_REPO_ROOT
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/r04j/trace_bimodal -o run -- python3 $R/scripts/prof_one.py bimodal 10 > $R/gpurun_out/r04j/trace_bimodal.log 2>&1) || exit 1
bash scripts/gpu_session.sh r04j pmc:main:uniform:FETCH_SIZE pmc:saltt:uniform:FETCH_SIZE bench || exit 1
