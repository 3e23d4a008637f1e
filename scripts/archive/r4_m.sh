#!/bin/bash
# round 4, GPU call M: split-K of the lm_head dgrad through the vocabulary (96 tiles of 256^2 at GPT-2
# small: split 2 = 192 blocks leaves 64 CUs idle; split 8 = 768 blocks = 3 whole rounds)
set -u
export TMPDIR=/tmp
rm -f gpurun_out/ab/summary.log
ROUNDS=3 STEPS=30 bash scripts/ab_bench.sh "" "DTC_VOCAB_SPLIT=8" "DTC_VOCAB_SPLIT=16" "DTC_VOCAB_SPLIT=4" || exit 1
cp gpurun_out/ab/summary.log gpurun_out/r4m_ab.log
