#!/bin/bash
# Round 5: strong C4 model, strips balanced with the all-to-all priced at 64 / 153 GB/s per link
set -o pipefail
OUT=gpurun_out
mkdir -p $OUT
timeout -k 10 500 python tools/strong_model.py --ranks 8 --balance-link 64 > $OUT/r05g_strong_model_c4_bal64.json 2> $OUT/r05g_bal64.err && echo "model 64 ok" &&
timeout -k 10 500 python tools/strong_model.py --ranks 8 --balance-link 153 > $OUT/r05g_strong_model_c4_bal153.json 2> $OUT/r05g_bal153.err && echo "model 153 ok"
