timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r5l_smoke.log 2>&1 && tail -1 gpurun_out/r5l_smoke.log \
&& scripts/gpu.sh test r5l_all tests -m gpu -rs
