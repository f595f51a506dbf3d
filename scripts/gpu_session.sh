#!/bin/bash
# One GPU-box session, parameterised (replaces the per-session scripts of rounds 1-3):
#
#   bash scripts/gpu_session.sh TAG STEP [STEP ...]
#
# Results go to gpurun_out/TAG/.  Every GPU step has its own time limit and the
# first failure ends the script (no retries).  Steps:
#   test            the whole GPU suite (pytest -m gpu)
#   test:EXPR       GPU tests matching -k EXPR
#   smoke           __graft_entry__.smoke()
#   bench           bench.py (the driver's default line)
#   trace           rocprofv3 --kernel-trace of the bench command (per-dispatch CSV + stats)
#   collect         PMC traffic + kernel-trace stats (scripts/collect_profiles.sh TAG)
#   aux             (f)-row rates (scripts/aux_bench.py)
#   auxpmc          VALU counters of the (f)-row kernels
#   host            host-to-host rates (scripts/host_bench.py)
#   pmc:LIB:WL:CTR  one rocprofv3 --pmc pass (counter CTR) of scripts/prof_one.py WL with the
#                   library main or ab_builds/libhyobfs_LIB.so
#   clk:WL:K:PT     per-dispatch GPU clock: rocprofv3 --pmc GRBM_COUNT GRBM_GUI_ACTIVE --kernel-trace
#                   of scripts/prof_one.py WL K (PT=1: output buffers pre-touched); scripts/clock_trace.py
#   clkbench:W      the same counters over the bench command (bench.py --steps 20 --warmup W)
#   kt:WL:K         rocprofv3 --kernel-trace --stats of scripts/prof_one.py WL K (per-kernel times)
#   udp:M:P:T:W[:R] tools/udp_bench M P 4 1200 1024 T W R (loopback PacketConn rate; M = batch|raw|coalesce|single;
#                   R = offered datagrams/s, 0 or absent = saturated)
#   bsq:KERN:SUF    SQ/TCC counter groups of the configs[2] batch under kernel KERN (pmc_bimodal_sq.sh)
#   ab              in-process A/B of library builds (scripts/ab_variants.py; AB_* env vars)
#   abg             the same for Gecko builds (scripts/ab_gecko_variants.py)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$(pwd)
TAG=${1:?tag}
shift
O=$R/gpurun_out/$TAG
mkdir -p "$O"
# the shipped library must be built from these sources (its build id is the source hash)
SHA=$(python3 scripts/src_sha.py)
grep -q "$SHA" hysteria_amd/libhyobfs.so || { echo "libhyobfs.so is not built from these sources ($SHA): rebuild"; exit 3; }
exec 3>&1   # step markers go to the session's stdout, not into a step's redirected output
step() {
  local name=$1 lim=$2; shift 2
  echo "== $name $(date +%T)" >&3
  timeout -k 10 "$lim" "$@"
  local rc=$?
  echo "== $name rc=$rc" >&3
  [ $rc -eq 0 ] || exit $rc
}
for s in "$@"; do
  case $s in
    test) step test 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread \
            > "$O/pytest_gpu.log" 2>&1 ;;
    test:*) step test 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread \
            -k "${s#test:}" > "$O/pytest_gpu_k.log" 2>&1 ;;
    smoke) step smoke 300 python -u -c "import __graft_entry__ as g; g.smoke()" > "$O/smoke.log" 2>&1 ;;
    bench) step bench 300 python -u bench.py > "$O/bench.json" 2> "$O/bench.err" ;;
    trace) (cd /tmp && export TMPDIR=/tmp && step trace 300 rocprofv3 --kernel-trace --stats --output-format csv \
            -d "$O/trace" -o run -- python3 "$R/bench.py" --steps 20 --warmup 5 --no-cpu-baseline --no-parity \
            > "$O/trace.log" 2>&1) || exit 1 ;;
    collect) step collect 1200 bash scripts/collect_profiles.sh "$TAG" > "$O/collect.log" 2>&1 ;;
    aux) step aux 300 python -u scripts/aux_bench.py > "$O/aux_bench.json" 2> "$O/aux_bench.err" ;;
    auxpmc) (cd /tmp && export TMPDIR=/tmp && step auxpmc 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_ACTIVE_INST_VALU \
            SQ_WAVES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --output-format csv -d "$O/pmc_aux" -o run -- \
            python3 "$R/scripts/aux_bench.py" > "$O/pmc_aux.log" 2>&1) || exit 1 ;;
    host) step host 600 python -u scripts/host_bench.py > "$O/host_bench.json" 2> "$O/host_bench.err" ;;
    pmc:*) IFS=: read -r _ LIBN WL CTR <<< "$s"
            LIBP=$R/hysteria_amd/libhyobfs.so
            [ "$LIBN" = main ] || LIBP=$R/ab_builds/libhyobfs_$LIBN.so
            (cd /tmp && export TMPDIR=/tmp && export HYOBFS_LIB=$LIBP && step "pmc $LIBN $WL $CTR" 240 rocprofv3 \
              --pmc $CTR --kernel-trace --output-format csv -d "$O/pmc_${LIBN}_${WL}_$CTR" -o run -- \
              python3 "$R/scripts/prof_one.py" "$WL" 5 > "$O/pmc_${LIBN}_${WL}_$CTR.log" 2>&1) || exit 1 ;;
    clk:*) IFS=: read -r _ WL K PT <<< "$s"
            (cd /tmp && export TMPDIR=/tmp && export PROF_PRETOUCH=$PT && step "clk $WL $K $PT" 240 rocprofv3 \
              --pmc GRBM_COUNT GRBM_GUI_ACTIVE --kernel-trace --output-format csv -d "$O/clk_${WL}_${K}_$PT" -o run -- \
              python3 "$R/scripts/prof_one.py" "$WL" "$K" > "$O/clk_${WL}_${K}_$PT.log" 2>&1) || exit 1 ;;
    clkbench:*) IFS=: read -r _ W <<< "$s"   # the bench command itself, W warmup steps
            (cd /tmp && export TMPDIR=/tmp && step "clkbench $W" 240 rocprofv3 \
              --pmc GRBM_COUNT GRBM_GUI_ACTIVE --kernel-trace --output-format csv -d "$O/clkbench_$W" -o run -- \
              python3 "$R/bench.py" --steps 20 --warmup "$W" --no-cpu-baseline --no-parity > "$O/clkbench_$W.log" 2>&1) || exit 1 ;;
    kt:*) IFS=: read -r _ WL K <<< "$s"
            (cd /tmp && export TMPDIR=/tmp && step "kt $WL $K" 240 rocprofv3 --kernel-trace --stats --output-format csv \
              -d "$O/kt_${WL}_$K" -o run -- python3 "$R/scripts/prof_one.py" "$WL" "$K" > "$O/kt_${WL}_$K.log" 2>&1) || exit 1 ;;
    udp:*) IFS=: read -r _ M P T W RATE <<< "$s"
            step "udp $M $P $T $W ${RATE:-0}" 120 tools/udp_bench "$M" "$P" 4 1200 1024 "$T" "$W" "${RATE:-0}" \
              > "$O/udp_${M}_${P}x${T}_w${W}_r${RATE:-0}.json" ;;
    bsq:*) IFS=: read -r _ KERN SUF <<< "$s"   # SQ/TCC counter groups of the configs[2] batch (scripts/pmc_bimodal_sq.sh)
            step "bsq $KERN" 700 bash scripts/pmc_bimodal_sq.sh "$KERN" "$SUF" > "$O/bsq_$KERN$SUF.log" 2>&1 ;;
    ab) step ab 600 python -u scripts/ab_variants.py ${AB_ARGS:-} > "$O/ab_${AB_NAME:-run}.txt" 2>&1 ;;
    abg) step abg 600 python -u scripts/ab_gecko_variants.py ${AB_ARGS:-} > "$O/abg_${AB_NAME:-run}.txt" 2>&1 ;;
    *) echo "unknown step $s"; exit 2 ;;
  esac
done
echo done
