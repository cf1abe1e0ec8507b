#!/bin/bash
# tools/gpu_ab.sh -- the one parameterised GPU runner for same-box A/B comparisons: library builds timed
# interleaved (tools/ab.py) and benchmark commands repeated per build.  Every A/B file under profiles/ has the
# invocation that reproduces it in profiles/README.md ("A/B index").
#
#   NAME=<tag>              results under gpurun_out/ab_<tag>/
#   VARIANTS="base v1 ..."  base = the shipped kcptube_amd/libkfec.so; any other name = kcptube_amd/variants/libkfec_<name>.so,
#                           built on the CPU beforehand by `python tools/build_variant.py <name> KEY=VAL ...` (compile-time
#                           knobs) or `tools/build_rev.sh <git-rev> libkfec_<name>` (an older revision); a ":ENV=VAL,..."
#                           suffix runs that build with extra environment (e.g. base:KFEC_QUEUE_PREFETCH=0)
#   TESTS="pytest files"    run against every non-base variant first: parity before timing
#   SHAPES="K:N:B:G[:erase[:pitch]] ..."
#                           coder shapes timed interleaved by tools/ab.py (erase: data | random | none | iid:<ppm>, as
#                           tools/ab_one.py's AB_ERASE; pitch: AB_PITCH)
#   CMD="command"           run once per round and variant with KFEC_LIB set (e.g. "python -u tools/bench_aead.py --steps 5",
#                           "./tools/latency_bench"); stdout to <variant>_r<round>.out
#   ROUNDS=3  LIMIT=400     interleaved rounds; time limit (s) of each GPU step
#
# Example (profiles/r05_xcd_span_ab.txt):
#   NAME=xcd VARIANTS="base xcd2 xcd4 xcd16" TESTS=tests/test_gpu_parity.py \
#     SHAPES="20:23:1440:1048576 10:13:1400:1048576:random 8:12:1440:1048576" tools/gpu_ab.sh
set -o pipefail
NAME=${NAME:-ab}; ROUNDS=${ROUNDS:-3}; LIMIT=${LIMIT:-400}
out=gpurun_out/ab_$NAME; mkdir -p $out
V=kcptube_amd/variants
lib_of() {  # variant spec -> library path (with the :ENV suffix kept for tools/ab.py)
  local name=${1%%:*} env=""
  [[ "$1" == *:* ]] && env=":${1#*:}"
  if [ "$name" = base ]; then echo "kcptube_amd/libkfec.so$env"; else echo "$V/libkfec_$name.so$env"; fi
}
env_of() {  # variant spec -> "KEY=VAL ..." for env(1)
  [[ "$1" == *:* ]] && echo "${1#*:}" | tr ',' ' '
}
for v in ${VARIANTS:-base}; do
  lib=$(lib_of "$v"); lib=${lib%%:*}
  [ -f "$lib" ] || { echo "missing $lib (build it on the CPU first: python tools/build_variant.py ...)"; exit 2; }
done
if [ -n "$TESTS" ]; then
  for v in ${VARIANTS:-base}; do
    [ "${v%%:*}" = base ] && continue
    lib=$(lib_of "$v"); lib=${lib%%:*}
    env KFEC_LIB=$lib $(env_of "$v") timeout -k 10 $LIMIT python -u -m pytest $TESTS -x -q --timeout 200 --timeout-method thread \
      > $out/tests_${v%%:*}.log 2>&1 || { tail -40 $out/tests_${v%%:*}.log; exit 1; }
    echo "${v%%:*}: $(tail -1 $out/tests_${v%%:*}.log)"
  done
fi
libs=""; for v in ${VARIANTS:-base}; do libs="$libs $(lib_of "$v")"; done
for s in $SHAPES; do
  IFS=: read -r K N B G E P X <<< "$s"
  if [ "$E" = iid ]; then E="iid:$P"; P=$X; fi  # (the erase field iid:<ppm> holds a colon itself)
  tag="${K}_${N}_${B}_${E:-data}${P:+_p$P}"
  AB_ERASE=${E:-data} AB_PITCH=${P:-0} timeout -k 10 $LIMIT python tools/ab.py $ROUNDS $libs -- $K $N $B $G > $out/ab_$tag.txt || { cat $out/ab_$tag.txt; exit 1; }
  echo "== $s"; cut -c1-160 $out/ab_$tag.txt
done
if [ -n "$CMD" ]; then
  for r in $(seq 1 $ROUNDS); do
    for v in ${VARIANTS:-base}; do
      lib=$(lib_of "$v"); lib=${lib%%:*}
      env KFEC_LIB=$([ "${v%%:*}" = base ] || echo $lib) $(env_of "$v") timeout -k 10 $LIMIT $CMD \
        > $out/${v%%:*}_r$r.out 2> $out/${v%%:*}_r$r.err || { tail -20 $out/${v%%:*}_r$r.err; exit 1; }
      echo "$r ${v%%:*}: $(tail -c 300 $out/${v%%:*}_r$r.out | tail -1)"
    done
  done
fi
echo ab-done
