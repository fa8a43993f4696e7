export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -s KILL 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_WAVES SQ_BUSY_CYCLES -d $PWD/gpurun_out/ttpmc -o ttpmc --output-format csv -- python3 tools/timetrack/run_timetrack.py --reps 2 > gpurun_out/ttpmc.json 2> gpurun_out/ttpmc.err; echo "pmc rc $?"
