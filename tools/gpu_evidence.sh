#!/bin/bash
# GPU evidence runner: every measurement this repo commits under profiles/ is produced by one of these subcommands,
# run on the MI355X box through gpurun (output under gpurun_out/<tag>/; every GPU step under its own time limit,
# steps chained so the first failure ends the call).
#
#   tools/gpu_evidence.sh suite    <tag> [pytest selection...]   -m gpu tests (default: the whole suite) + smoke()
#   tools/gpu_evidence.sh bench    <tag> [config...]              no config: the driver's default line (c4 + configs
#                                                                 block + parity); else one short line per config
#   tools/gpu_evidence.sh perstep  <tag> <config> [S1 S2]         per-step rocprofv3 kernel table: two --kernel-trace
#                                                                 --stats runs differing in timed steps, differenced
#                                                                 by tools/prof_diff.py (set-up / warmup cancel)
#   tools/gpu_evidence.sh traffic  <tag> <config> [family]        HBM bytes of a kernel family (gemm | mfma | gn | loss)
#                                                                 over one step: FETCH_SIZE and WRITE_SIZE in separate
#                                                                 --pmc passes, gfx950 correction in pmc_traffic.py
#   tools/gpu_evidence.sh pmc      <tag> <shape> <pass> <prec>    conv counter sets (MFMA busy, waits, VALU / SALU /
#                                                                 LDS issue) of one tools/conv_bench.py shape + pass
#   tools/gpu_evidence.sh pmcrun   <tag> <name> <regex> <cmd...>  the same counter sets over any program (the kernels
#                                                                 matching regex; settings through exported env vars)
#   tools/gpu_evidence.sh ab       <tag> <config> <variant...>    interleaved A/B of library builds variants/<v>/
#                                                                 (tools/build_variant.sh), "default" (in-tree) or
#                                                                 "env:VAR=VAL[,...]" (in-tree under those settings)
#   tools/gpu_evidence.sh loops    <tag> <variant...>              interleaved A/B of library builds on the GEMM main
#                                                                 loops: tools/loop_bench.py (plain 4k GEMM + c4 3x3
#                                                                 layers) and tools/dma_exp.py (per-pass conv), both
#                                                                 arithmetics ("default" = the in-tree library)
#   tools/gpu_evidence.sh final    <tag>                          round-end set: suite + smoke, default bench line,
#                                                                 per-step tables of c3 and c4
set -o pipefail
CMD=$1; TAG=${2:-t}; shift 2
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/$TAG
mkdir -p $OUT

suite() {
  local sel=("$@")
  [ ${#sel[@]} -eq 0 ] && sel=(tests)
  timeout -k 10 1000 python -u -m pytest "${sel[@]}" -m gpu -v --timeout 300 --timeout-method thread \
    > $OUT/pytest.log 2>&1
  local rc=$?
  grep -E "FAILED|ERROR" $OUT/pytest.log | head -20; tail -2 $OUT/pytest.log
  [ $rc -eq 0 ] || return $rc
  timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $OUT/smoke.log 2>&1 \
    || return $?
  tail -1 $OUT/smoke.log
}

bench() {
  if [ $# -eq 0 ]; then
    timeout -k 10 600 python -u bench.py --detail-out $OUT/bench_detail.json > $OUT/bench.json 2> $OUT/bench.err || return $?
    cut -c1-600 $OUT/bench.json
    return 0
  fi
  for c in "$@"; do
    timeout -k 10 400 python -u bench.py --config $c --steps 10 --warmup 3 --no-cpu-baseline --detail \
      --detail-out $OUT/bench_${c}_detail.json > $OUT/bench_$c.json 2> $OUT/bench_$c.err || return $?
    python3 tools/bench_brief.py $OUT/bench_$c.json $c
  done
}

perstep() {
  local cfg=$1 s1=${2:-} s2=${3:-}
  case $cfg in c4|c5) s1=${s1:-1}; s2=${s2:-3};; *) s1=${s1:-2}; s2=${s2:-12};; esac
  for s in $s1 $s2; do
    timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/prof_${cfg}_s$s -o run --output-format csv -- \
      python3 bench.py --config $cfg --steps $s --warmup 1 --no-cpu-baseline --no-kernel-timing --no-parity \
      > $OUT/prof_${cfg}_s$s.log 2>&1 || return $?
  done
  python3 tools/prof_diff.py $OUT/prof_${cfg}_s$s1 $OUT/prof_${cfg}_s$s2 $((s2 - s1)) > $OUT/prof_${cfg}_per_step.txt \
    || return $?
  head -30 $OUT/prof_${cfg}_per_step.txt | cut -c1-160
}

traffic() {
  local cfg=$1 fam=${2:-gemm} re
  case $fam in gemm) re=gemm3x;; gn) re=gn_;; mfma) re=$(python3 -c "import sys; sys.path.insert(0, 'tools'); from frac_from_prof import FAMILY; print(FAMILY.pattern)");; loss) re="reparam_|reduce_partial|reduce_final|kl_bwd|recon_bwd";;
    *) echo "family: gemm | mfma | gn | loss"; return 2;; esac
  for c in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 400 rocprofv3 --pmc $c --kernel-include-regex "$re" -d gpurun_out/traffic_${cfg}_${fam}_$c -o run \
      --output-format csv -- python3 bench.py --config $cfg --steps 1 --warmup 0 --no-cpu-baseline \
      --no-kernel-timing --no-parity > $OUT/traffic_${cfg}_${fam}_$c.log 2>&1 || return $?
  done
  python3 tools/pmc_traffic.py $cfg $TAG $fam || return $?
  mkdir -p $OUT/profiles && cp profiles/${TAG}_${cfg}_*traffic.json $OUT/profiles/ 2>/dev/null
  return 0
}

PMC_SETS=(
 "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_INSTS_MFMA"
 "SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE SQ_BUSY_CU_CYCLES SQ_ACTIVE_INST_SCA SQ_INSTS_SALU"
)
pmc() {
  local shape=$1 pass=$2 prec=${3:-32} i=0
  for set in "${PMC_SETS[@]}"; do
    local o=$OUT/s${shape}_${pass}_${prec}_$i
    timeout -s KILL 120 rocprofv3 --pmc $set --kernel-include-regex gemm3x -d $o -o run --output-format csv -- \
      python3 tools/one_conv.py --shape $shape --pass_ $pass --reps 3 --precision $prec > $o.log 2>&1 || return $?
    i=$((i + 1))
  done
  echo "== shape $shape $pass $prec"
  python3 tools/pmc_summary.py "$OUT/s${shape}_${pass}_${prec}_*/**/*counter_collection.csv"
}

pmcrun() {
  local name=$1 re=$2 i=0; shift 2
  for set in "${PMC_SETS[@]}"; do
    timeout -s KILL 120 rocprofv3 --pmc $set --kernel-include-regex "$re" -d $OUT/${name}_$i -o run --output-format csv \
      -- "$@" > $OUT/${name}_$i.log 2>&1 || return $?
    i=$((i + 1))
  done
  echo "== $name"
  python3 tools/pmc_summary.py "$OUT/${name}_*/**/*counter_collection.csv"
}

ab() {
  local cfg=$1; shift
  for r in 1 2; do
    for v in "$@"; do
      local lib=variants/$v/libmvae_hip.so envs=() tag=${v//[:=,]/_}
      [ "$v" = default ] && lib=medvae_disentangled_multimodal_amd/libmvae_hip.so
      # "env:VAR=VAL[,VAR=VAL]": the in-tree library under those environment settings
      if [[ $v == env:* ]]; then lib=medvae_disentangled_multimodal_amd/libmvae_hip.so; IFS=, read -ra envs <<< "${v#env:}"; fi
      env "${envs[@]}" MVAE_HIP_LIB=$lib timeout -k 10 300 python -u bench.py --config $cfg --steps 6 --warmup 2 \
        --no-cpu-baseline --detail --detail-out $OUT/ab_${cfg}_${tag}_${r}_detail.json > $OUT/ab_${cfg}_${tag}_$r.json 2> $OUT/ab_${cfg}_${tag}_$r.err || return $?
      python3 tools/bench_brief.py $OUT/ab_${cfg}_${tag}_$r.json "$v"
    done
  done
}

loops() {
  for r in 1 2; do
    for v in "$@"; do
      local lib=variants/$v/libmvae_hip.so envs=()
      [ "$v" = default ] && lib=medvae_disentangled_multimodal_amd/libmvae_hip.so
      # "env:VAR=VAL[,VAR=VAL]": the in-tree library under those environment settings
      if [[ $v == env:* ]]; then lib=medvae_disentangled_multimodal_amd/libmvae_hip.so; IFS=, read -ra envs <<< "${v#env:}"; fi
      for p in ${PRECS:-bf16-mixed 32}; do
        echo "== $v $p" >> $OUT/loops.txt
        env "${envs[@]}" MVAE_HIP_LIB=$lib timeout -k 10 200 python -u tools/loop_bench.py $p >> $OUT/loops.txt 2>> $OUT/loops.err || return $?
        env "${envs[@]}" MVAE_HIP_LIB=$lib timeout -k 10 200 python -u tools/dma_exp.py $p >> $OUT/loops.txt 2>> $OUT/loops.err || return $?
      done
    done
  done
  cat $OUT/loops.txt
}

case $CMD in
  suite) suite "$@" ;;
  bench) bench "$@" ;;
  perstep) perstep "$@" ;;
  traffic) traffic "$@" ;;
  pmc) pmc "$@" ;;
  pmcrun) pmcrun "$@" ;;
  ab) ab "$@" ;;
  loops) loops "$@" ;;
  final) suite && bench && perstep c3 && perstep c4 ;;
  *) echo "unknown subcommand $CMD"; exit 2 ;;
esac
