#!/bin/bash
# One bench.py configuration under each value of environment knobs, either
# timed (bench line only), kernel-traced (rocprofv3 --kernel-trace --stats) or
# counter-sampled (one rocprofv3 --pmc pass per variant).  Replaces round 2-5's
# one-off probes (tools/probe/*: hand-off rounds, stretch packing, mirrored
# lanes, icache / clock / stretch counters, C5 layouts, packed problems per wave).
#   TAG=rounds ARGS="--collision" VARIANTS="IKG_HANDOFF_ROUNDS=0 IKG_HANDOFF_ROUNDS=2" MODE=trace tools/knob_trace.sh
#   TAG=icache ARGS="--collision --steps 2 --warmup 1" VARIANTS="IKG_HANDOFF_ROUNDS=1,IKG_STRETCH_PPW=1 \
#       IKG_HANDOFF_ROUNDS=1,IKG_STRETCH_PPW=32" MODE="pmc:SQ_WAVES SQ_IFETCH SQC_ICACHE_HITS SQC_ICACHE_MISSES" tools/knob_trace.sh
#   TAG=c5v ARGS="--dtype f32 --batch 512 --multistart 256" VARIANTS="base" EXTRA="--variant 0|--variant 1|--variant 2" tools/knob_trace.sh
# A variant is NAME=VALUE[,NAME=VALUE...] or "base"; EXTRA is a |-separated
# list of further bench.py argument sets (each run under every variant).
# Outputs: gpurun_out/$TAG/<variant>[_<extra#>].json (+ rocprof dirs), and a
# one-line-per-run summary in gpurun_out/$TAG/summary.txt.  Every GPU step has
# its own time limit; a failing step ends the script.
TAG=${TAG:?TAG=name}
R=$(pwd); O=$R/gpurun_out/$TAG; mkdir -p $O
export TMPDIR=/tmp
MODE=${MODE:-time}
IFS='|' read -r -a EXTRAS <<< "${EXTRA:-}"
[ ${#EXTRAS[@]} -eq 0 ] && EXTRAS=("")
for rep in $(seq 1 ${REPS:-1}); do
  for v in ${VARIANTS:-base}; do
    envs=$( [ "$v" = base ] || echo $v | tr ',' ' ')
    for i in "${!EXTRAS[@]}"; do
      n=${v//[=,]/_}_x${i}_r$rep
      args="--no-cpu-baseline --no-extra ${ARGS:-} ${EXTRAS[$i]}"
      case $MODE in
        time) (cd $R && env $envs timeout -k 10 ${LIMIT:-240} python bench.py $args > $O/$n.json 2> $O/$n.err) ;;
        trace) (cd /tmp && env $envs timeout -k 10 ${LIMIT:-240} rocprofv3 --kernel-trace --stats --output-format csv \
                  -d $O/$n -o run -- python3 $R/bench.py $args > $O/$n.json 2> $O/$n.err) ;;
        pmc:*) (cd /tmp && env $envs timeout -s KILL ${LIMIT:-90} rocprofv3 --pmc ${MODE#pmc:} --output-format csv \
                  -d $O/$n -o run -- python3 $R/bench.py $args > $O/$n.json 2> $O/$n.err) ;;
        *) echo "unknown MODE $MODE"; exit 2 ;;
      esac
      rc=$?; [ $rc -eq 0 ] || { echo "FATAL $n rc=$rc"; tail -3 $O/$n.err; exit $rc; }
      python3 -c "import json; d=json.load(open('$O/$n.json')); print('$n', round(d['ms_per_step'], 4), 'ms/step', round(d['roofline'].get('kernel_ms', 0), 4), 'kernel ms')" | tee -a $O/summary.txt
    done
  done
done
echo ALLDONE
