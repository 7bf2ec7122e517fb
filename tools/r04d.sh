#!/bin/bash
# r04d GPU session: copy floors of the intermediate layouts, the 512^3 chunking probe and the
# 3-sweep shape A/B (bench + rocprof per shape).
set -e
OUT=${GRAFT_REPO_ROOT:-$PWD}/gpurun_out
timeout -k 10 120 python tools/kexp/run_seg_chain.py > $OUT/r04d_seg_chain.txt 2>&1
timeout -k 10 240 python tools/probe_512_chunk.py 512 > $OUT/r04d_probe512.jsonl 2>&1
bash tools/ab_blocked.sh r04d
