C="--config c4 --c4-calls 3000 --steps 2 --warmup 0 --cpu-sample 0"
P='import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); s=d["split_last_step"]; print(sys.argv[2], round(s["wall_ms"]), s["phases_ms"].get("hist_apply"), s["phases_ms"].get("timers"))'
scripts/gpu.sh bench r5e_a $C && python3 -c "$P" gpurun_out/r5e_a.json pf1 \
&& SH_HIST_PF=0 scripts/gpu.sh bench r5e_b $C && python3 -c "$P" gpurun_out/r5e_b.json pf0 \
&& scripts/gpu.sh bench r5e_c $C && python3 -c "$P" gpurun_out/r5e_c.json pf1 \
&& SH_HIST_PF=0 scripts/gpu.sh bench r5e_d $C && python3 -c "$P" gpurun_out/r5e_d.json pf0 \
&& scripts/gpu.sh test r5e_c4 tests/test_gpu_c4.py tests/test_gpu_snapshot.py tests/test_gpu_shard_stream.py
