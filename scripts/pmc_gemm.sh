#!/bin/bash
# SQ counter passes over single GEMM shapes of scripts/bench_gemm_f32.py
# usage: bash scripts/pmc_gemm.sh <shape[,shape]> <tile|auto> <outdir>
set -u
shape=$1; tile=$2; out=$3
mkdir -p "$out"
P1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU SQ_LDS_BANK_CONFLICT"
P2="SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_VMEM SQ_WAIT_INST_LDS SQ_LDS_IDX_ACTIVE SQ_INSTS_SALU GRBM_GUI_ACTIVE GRBM_COUNT"
envs="GEMM_ONLY=$shape"
[ "$tile" != auto ] && envs="$envs MOG_GEMM_TILE=$tile"
i=0
for P in "$P1" "$P2"; do
  i=$((i+1))
  env $envs timeout -s KILL 90 rocprofv3 --pmc $P --output-format csv -d "$out/p$i" -o run -- python3 scripts/bench_gemm_f32.py > "$out/p$i.log" 2>&1 || { echo "pass $i failed"; exit 1; }
done
echo ok
