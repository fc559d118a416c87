timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r4y_smoke.log 2>&1 && tail -3 gpurun_out/r4y_smoke.log \
&& scripts/gpu.sh test r4y_all tests -m gpu -rs
