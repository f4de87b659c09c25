#!/usr/bin/env bash
# A/B of round-kernel variants (tools/ab/libpsim_<name>.so, built with
# `make -C partisan_amd/csrc variant NAME=<name> DEFS=...`) against the product
# libpsim.so ("cur"): bench.py's timed steps, sustained rate and per-round
# table for each, interleaved so box drift hits every variant alike.
# A variant may carry one environment setting: cur@PSIM_DENSE_DIV=16.
#   VARIANTS="cur gs2 cur gs2" bash tools/ab/gs_ab.sh
set -u
mkdir -p gpurun_out/ab
for spec in ${VARIANTS:-cur gs2 gs2f gs3 cur gs2 gs2f gs3}; do
  v=${spec%%@*}; envset=""; [ "$spec" != "$v" ] && envset=${spec#*@}
  if [ "$v" = cur ]; then lib=$PWD/partisan_amd/libpsim.so; else lib=$PWD/tools/ab/libpsim_$v.so; fi
  tag=$(echo "$spec" | tr '@=' '__')
  k=$(ls gpurun_out/ab | grep -c "^${tag}_[0-9]" || true)
  log=gpurun_out/ab/${tag}_$k.log
  env $envset PSIM_LIB_PATH=$lib timeout -k 10 240 python bench.py --steps 20 --warmup 3 --no-cpu-baseline \
      --no-parity --sustain-s 2 > "$log" 2>&1 || { echo "variant $spec failed: $?"; tail -5 "$log"; exit 1; }
  python3 - "$log" "$spec" <<'EOF'
import json, sys
d = [json.loads(x) for x in open(sys.argv[1]) if x.startswith("{")][-1]
rl = d["roofline"]
us = " ".join(f"{r['us']:.0f}" for r in rl["per_round"])
print(f"{sys.argv[2]:>22} ms/step {d['ms_per_step']:.3f} sustained {d['sustained']['ms_per_step']:.3f} "
      f"frac {rl['frac']:.3f} | per-round us: {us}", flush=True)
EOF
done
