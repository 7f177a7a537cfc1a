#!/bin/bash
# quick A/B: parity subset on the first variant, then the bench A/B (tools/gpu_ab.sh)
# usage: LIBS="new base" WLS="config4 config3" tools/gpu_ab_quick.sh TAG
set -o pipefail
PARITY=${PARITY:-"512_thread or warp or hram"} tools/gpu_ab.sh "$1"
