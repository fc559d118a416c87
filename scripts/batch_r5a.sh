B="--config c2 --steps 20 --warmup 3 --cpu-sample 0 --no-verify"
SH_BK_SCAT=8 scripts/gpu.sh bench r5a_s8 --config c2 --steps 20 --warmup 3 --cpu-sample 0 \
&& scripts/gpu.sh bench r5a_s4 $B \
&& SH_BK_SCAT=8 scripts/gpu.sh bench r5a_s8b $B \
&& scripts/gpu.sh bench r5a_s4b $B \
&& SH_BK_SCAT=8 scripts/gpu.sh bench r5a_c3s8 --config c3 --steps 10 --warmup 2 --cpu-sample 0 \
&& scripts/gpu.sh bench r5a_c3s4 --config c3 --steps 10 --warmup 2 --cpu-sample 0 --no-verify
