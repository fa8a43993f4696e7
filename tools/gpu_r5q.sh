#!/bin/bash
# Round 5: strong C4 after the ragged planner changes
set -o pipefail
OUT=gpurun_out
mkdir -p $OUT
timeout -k 10 300 python bench.py --strong --steps 5 --warmup 2 > $OUT/r05q_strong.json 2> $OUT/r05q_strong.err && echo "strong ok" &&
timeout -k 10 500 python tools/strong_model.py --ranks 8 > $OUT/r05q_strong_model_c4.json 2> $OUT/r05q_model.err && echo "model ok"
