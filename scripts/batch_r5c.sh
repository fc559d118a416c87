B="--config c2 --steps 20 --warmup 3 --cpu-sample 0 --no-verify"
X="SH_BK_SPAN=2048 SH_BK_CH=1024 SH_BK_MINB=8"
Y="SH_BK_SPAN=2048 SH_BK_CH=1536 SH_BK_MINB=8"
scripts/gpu.sh bench r5c_def $B \
&& env $X scripts/gpu.sh bench r5c_x $B \
&& env $Y scripts/gpu.sh bench r5c_y $B \
&& scripts/gpu.sh bench r5c_def2 $B \
&& env $X scripts/gpu.sh bench r5c_x2 $B \
&& env $Y scripts/gpu.sh bench r5c_y2 $B
