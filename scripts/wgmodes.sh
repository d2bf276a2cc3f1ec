#!/bin/bash
# A/B of wgrad_tn_bf16_kernel forms (profiling build: MOG_WG_MODE loader /
# probes, MOG_WG_MAP split->XCD mapping) and layer subsets, HIP-event times
R=$GRAFT_REPO_ROOT
export MOG_AIR_LIB=$R/mog-asr_amd/mog_air/_lib/prof/libmog_air.so WG_ONLY_NEW=1
run() { env "$@" timeout -k 10 120 python3 $R/scripts/wgrad_shapes.py 2>&1 | grep variant || exit 1; }
run WG_SPLITS=8,16,24 MOG_WG_MODE=0
run WG_SPLITS=8,16 MOG_WG_MODE=2
run WG_SPLITS=8 MOG_WG_MODE=3
run WG_SPLITS=8 MOG_WG_MODE=4
