#!/bin/bash
# The one GPU call runner (sent as: gpurun -- 'bash tools/gpu_runs/run.sh MODE LABEL ...').
# Every GPU step runs under its own time limit (tools/gpu_steps.sh or timeout -k),
# and the call stops at the first step that timed out, aborted or crashed.
# Logs and JSON lines land in gpurun_out/<label>_*; the summaries kept are copied
# into profiles/ (README.md: which call produced which committed file).
#
#   run.sh tests LABEL [PYTEST_ARGS...]       GPU suite (default: tests -m gpu) + smoke
#   run.sh ab LABEL REPS "LIB..." [BENCH_ARGS...]
#                                             A/B bench of variant libraries (lib/libbdpt_amd_<LIB>.so,
#                                             "default" = the product library; LIB:VAR=v,VAR2=w also sets
#                                             environment for that run), REPS alternating passes,
#                                             one summary line per run in gpurun_out/LABEL.txt
#   run.sh abtest LABEL "LIB..." [PYTEST_FILES...]
#                                             parity suites on variant libraries before an A/B
#   run.sh profile LABEL SCENE W H SPP        kernel trace + stamped PMC passes (tools/profile_round.sh)
#   run.sh final LABEL                        suite, smoke, the stamped PMC profiles of the four
#                                             BASELINE workloads, then every bench line, each bench
#                                             under rocprofv3 --kernel-trace --stats, so a line and its
#                                             kernel CSV come from the same run
#   run.sh final_a / final_c / final_b LABEL  the same in three calls (a call is limited to 20 minutes;
#                                             final_tc = final_a's suite + smoke, then final_c):
#                                             suite + smoke + the 512^2 PMC profiles; the 1024^2 and
#                                             synth1m profiles; the bench lines (copy each call's
#                                             gpurun_out/prof_LABEL/pmc_*.json into profiles/ between)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
MODE=$1 LABEL=$2
shift 2
L=$PWD/bidirectional-path-tracing_amd/lib
mkdir -p gpurun_out

lib_path() { [ "$1" = default ] && echo "$L/libbdpt_amd.so" || echo "$L/libbdpt_amd_$1.so"; }

summary() {  # label json -> one line: label value ms_per_step counts
  python3 - "$1" "$2" <<'PY'
import json, sys
d = json.loads(open(sys.argv[2]).read().strip().splitlines()[-1])
c = (d.get("roofline") or {}).get("counts_per_sample") or {}
p = (d.get("parity") or {}).get("max_rel_l2")
eff = {}
if c.get("trav_wave_iters"):
    eff["trav_simd"] = c["trav_lane_iters"] / c["trav_wave_iters"] / 64
if c.get("shade_wave_actions"):
    eff["shade_simd"] = c["shade_lane_actions"] / c["shade_wave_actions"] / 64
print(sys.argv[1], d["value"], d["ms_per_step"], "parity", p,
      " ".join(f"{k}={c[k]:.4g}" for k in ("interior_visits", "tri_tests", "loop_clocks", "trav_clocks", "shade_clocks",
                                            "trav_wave_iters", "shade_wave_actions") if k in c),
      " ".join(f"{k}={v:.3f}" for k, v in eff.items()),
      "sched", (d.get("roofline") or {}).get("sched_per_sample"))
PY
}

case $MODE in
tests)
  ARGS=("$@")
  [ ${#ARGS[@]} -eq 0 ] && ARGS=(tests -m gpu)
  tools/gpu_steps.sh \
    "500 ${LABEL}_gpu_tests.log -- python -u -m pytest ${ARGS[*]} -x -q --timeout 300 --timeout-method thread" \
    "120 ${LABEL}_smoke.log -- python -c 'import __graft_entry__ as g; g.smoke(); print(\"smoke ok\")'"
  ;;
abtest)
  LIBS=$1; shift
  FILES=("$@")
  [ ${#FILES[@]} -eq 0 ] && FILES=(tests/test_gpu_parity.py tests/test_gpu_kat.py)
  for lib in $LIBS; do
    BDPT_AMD_LIB=$(lib_path $lib) timeout -k 10 400 python -u -m pytest "${FILES[@]}" -x -q --timeout 200 \
      --timeout-method thread > gpurun_out/${LABEL}_tests_$lib.log 2>&1
    rc=$?
    tail -1 gpurun_out/${LABEL}_tests_$lib.log
    if [ $rc -ne 0 ]; then exit $rc; fi
  done
  ;;
ab)
  REPS=$1 LIBS=$2; shift 2
  : > gpurun_out/$LABEL.txt
  for rep in $(seq 1 $REPS); do
    for lib in $LIBS; do
      # LIB may carry environment settings for the run: name:VAR=v,VAR2=w
      name=${lib%%:*} envs=""
      [ "$name" != "$lib" ] && envs=${lib#*:}
      tag=$(echo "$lib" | tr ':=,' '_-_')
      out=gpurun_out/${LABEL}_${tag}_$rep.json
      env ${envs//,/ } BDPT_AMD_LIB=$(lib_path $name) timeout -k 10 300 python3 bench.py --no-cpu --no-parity "$@" > $out 2> ${out%.json}.err
      rc=$?
      if [ $rc -ne 0 ]; then echo "$lib rep $rep rc=$rc" >> gpurun_out/$LABEL.txt; tail -5 ${out%.json}.err; exit $rc; fi
      summary ${tag}_$rep $out | tee -a gpurun_out/$LABEL.txt
    done
  done
  ;;
profile)
  timeout -k 10 900 bash tools/profile_round.sh $LABEL "$@"
  ;;
final|final_a|final_b|final_c|final_tc|final_pc|final_ac)
  P=gpurun_out/prof_$LABEL
  kt() {  # name limit bench args...: the bench line under the kernel trace
    local name=$1 lim=$2; shift 2
    echo "$lim ${LABEL}_bench_$name.json -- rocprofv3 --kernel-trace --stats -d $P/kt_$name -o kt --output-format csv -- python3 bench.py $*"
  }
  A=( \
    "500 ${LABEL}_gpu_tests.log -- python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread" \
    "120 ${LABEL}_smoke.log -- python -c 'import __graft_entry__ as g; g.smoke(); print(\"smoke ok\")'" \
    "300 ${LABEL}_prof_caustic.log -- bash tools/profile_round.sh $LABEL caustic 512 512 256" \
    "300 ${LABEL}_prof_hl.log -- bash tools/profile_round.sh $LABEL hardlight 512 512 1024" )
  C=( \
    "400 ${LABEL}_prof_c1024.log -- bash tools/profile_round.sh $LABEL caustic 1024 1024 1024" \
    "500 ${LABEL}_prof_synth.log -- bash tools/profile_round.sh $LABEL synth1m 2048 2048 512" )
  CP=( "30 ${LABEL}_copy.log -- cp $P/pmc_*.json profiles/ && ls -la profiles/pmc_*" )
  # (final_b on another box: copy gpurun_out/prof_LABEL/pmc_*.json into profiles/ first, locally)
  B=( \
    "$(kt caustic_512x512_256spp 250 --steps 20 --warmup 2)" \
    "$(kt hardlight_512x512_1024spp 250 --scene hardlight --spp 1024 --steps 5 --warmup 1)" \
    "$(kt caustic_1024x1024_1024spp 300 --width 1024 --height 1024 --spp 1024 --steps 1 --warmup 1)" \
    "$(kt synth1m_2048x2048_512spp 400 --scene synth1m --width 2048 --height 2048 --spp 512 --steps 1 --warmup 1)" \
    "$(kt path_caustic_512x512_64spp 150 --integrator path --spp 64 --steps 5 --warmup 1)" \
    "$(kt direct_caustic_512x512_64spp 150 --integrator direct --spp 64 --steps 5 --warmup 1)" \
    "200 ${LABEL}_tail.log -- python3 tools/shard_tail.py caustic 512 512 256 1 8" \
    "$(kt rr_hardlight_512x512_1024spp 250 --russian-roulette --scene hardlight --spp 1024 --steps 2 --warmup 1 --count-spp 16)" \
    "$(kt rr_caustic_512x512_256spp 420 --russian-roulette --steps 1 --warmup 0)" )
  case $MODE in
  final) tools/gpu_steps.sh "${A[@]}" "${C[@]}" "${CP[@]}" "${B[@]}" ;;
  final_a) tools/gpu_steps.sh "${A[@]}" ;;
  final_c) tools/gpu_steps.sh "${C[@]}" ;;
  final_tc) tools/gpu_steps.sh "${A[0]}" "${A[1]}" "${C[@]}" ;;  # (suite + smoke, then final_c)
  final_ac) tools/gpu_steps.sh "${A[@]}" "${C[@]}" ;;  # (final_a then final_c)
  final_pc) tools/gpu_steps.sh "${A[1]}" "${A[2]}" "${A[3]}" "${C[@]}" ;;  # (smoke and all four profiles: the suite ran on the build already)
  final_b) tools/gpu_steps.sh "${B[@]}" ;;
  esac
  ;;
*)
  echo "usage: run.sh tests|abtest|ab|profile|final LABEL ..." >&2
  exit 2
  ;;
esac
