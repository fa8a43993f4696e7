export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 500 python -u tools/bench_rows.py --mode continuum --rows 390625 --nchan 256 --npix 4096 --facets-xy 8 4 --world 8 --refcall > gpurun_out/c5_ref.json 2> gpurun_out/c5_ref.err; echo "c5 ref rc $?"
timeout -k 10 500 python -u tools/bench_rows.py --mode continuum --rows 390625 --nchan 256 --npix 4096 --facets-xy 8 4 --world 8 > gpurun_out/c5_2d.json 2> gpurun_out/c5_2d.err; echo "c5 2d rc $?"
