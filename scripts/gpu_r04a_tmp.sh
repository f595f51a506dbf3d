set -u
R=$GRAFT_REPO_ROOT
mkdir -p gpurun_out/r04m
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/r04m/trace_alt -o run -- python3 $R/scripts/prof_one.py bimodal_alt 20 > $R/gpurun_out/r04m/trace_alt.log 2>&1) || exit 1
AB_ARGS="tile" AB_NAME=uniform bash scripts/gpu_session.sh r04m ab || exit 1
