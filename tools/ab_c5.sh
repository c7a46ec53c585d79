#!/bin/bash
# Config-5 A/B of libraries on one lease: A B A B, batch 1024 and 1 (tools/config5_prof.py,
# BA_HIP_LIB selects each library).  usage: bash tools/ab_c5.sh out.log libA libB ...
set -o pipefail
out=$1; shift
mkdir -p gpurun_out
for rep in 1 2; do for lib in "$@"; do for b in 1024 1; do
  echo "lib=$lib rep=$rep batch=$b $(BA_HIP_LIB=$PWD/$lib timeout -k 10 120 python tools/config5_prof.py --batch $b --reps 400 2>/dev/null | grep -o '"us_per_call[a-z_]*": [0-9.]*' | tr '\n' ' ')" | tee -a $out || exit 1
done; done; done
