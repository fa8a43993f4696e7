export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $PWD/gpurun_out/tt -o tt --output-format csv -- python3 tools/timetrack/run_timetrack.py --reps 5 > gpurun_out/tt.json 2> gpurun_out/tt.err; echo "tt rc $?"
python3 tools/kstats.py timetrack gpurun_out/tt > gpurun_out/tt_kstats.txt; echo "ks rc $?"
