#!/bin/bash
# Config-5 A/B on one lease: A B A B, batch 1024 and 1 (tools/config5_prof.py).
# Each variant is a library (BA_HIP_LIB selects it) or `env:NAME=VALUE` (the
# product library with that variable set, e.g. a per-call switch).
# usage: bash tools/ab_c5.sh out.log variantA variantB ... [-- batch ...]
set -o pipefail
out=$1; shift
vars=(); batches=(1024 1)
while [ $# -gt 0 ]; do
  if [ "$1" = "--" ]; then shift; batches=("$@"); break; fi
  vars+=("$1"); shift
done
mkdir -p gpurun_out
PROD=byzantine-agreement_amd/ba_amd/libba_hip.so
for rep in 1 2; do for v in "${vars[@]}"; do for b in "${batches[@]}"; do
  if [[ $v == env:* ]]; then lib=$PROD; ev=${v#env:}; else lib=$v; ev=BA_AB_NONE=1; fi
  echo "var=$v rep=$rep batch=$b $(env "$ev" BA_HIP_LIB=$PWD/$lib timeout -k 10 120 python tools/config5_prof.py --batch $b --reps 400 2>/dev/null | grep -o '"us_per_call[a-z_]*": [0-9.]*' | tr '\n' ' ')" | tee -a $out || exit 1
done; done; done
