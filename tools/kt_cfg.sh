#!/bin/bash
# GPU box: rocprofv3 kernel stats of bench.py under several launch policies
# (LPC_* environment), one run per config: kt_cfg.sh 'LPC_BUDGET=0' 'LPC_BUDGET=32' ...
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd /tmp && export TMPDIR=/tmp
i=0
for cfg in "$@"; do
  out=$R/gpurun_out/ktcfg/$i; mkdir -p $out
  echo "$cfg" > $out/cfg.txt
  env $cfg > /dev/null   # validate syntax
  if [ -n "$KT_SCENE" ]; then     # another scene: tools/sweep.py with the one config (KT_SCENE, KT_N)
    ( timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $out -o kt --output-format csv -- \
        python3 $R/tools/sweep.py $KT_SCENE ${KT_N:-1000000} 3 ${cfg//LPC_/} > $out/bench.log 2>&1 ) || { echo "cfg $cfg failed"; exit 1; }
  else
    ( export $cfg; timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $out -o kt --output-format csv -- \
        python3 $R/bench.py --steps 5 --warmup 1 --no-cpu > $out/bench.log 2>&1 ) || { echo "cfg $cfg failed"; exit 1; }
  fi
  i=$((i+1))
done
python3 $R/tools/kt_print.py $R/gpurun_out/ktcfg
