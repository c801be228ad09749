#!/bin/bash
# Attention kernel variants A/B (GPT-2-medium shape, B=64): tools/attn_probe.py under
# each env config (K=V[;K=V..]), 2 interleaved rounds.
#   bash tools/attn_ab.sh 'PDO_ATTN_FWDV=0;PDO_ATTN_DQV=0' 'PDO_ATTN_FWDV=3;PDO_ATTN_DQV=1'
set -o pipefail
for r in 1 2; do
  for cfg in "$@"; do
    out=$( (IFS=';'; for kv in $cfg; do export "$kv"; done
            timeout -k 10 180 python tools/attn_probe.py --B 64 2>/dev/null) ) || { echo "failed: $cfg"; exit 1; }
    echo "r$r [$cfg] $(echo "$out" | tail -1)"
  done
done
