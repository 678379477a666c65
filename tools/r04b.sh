C4="--sims 1600 --channels 256 --blocks 20 --steps 4 --warmup 1 --sustained-moves 0 --cpu-baseline-moves 0"
C5="--games 512 --dtype fp16 --eval-batch 2048 --steps 10 --warmup 2 --sustained-moves 0 --cpu-baseline-moves 0"
OUT=gpurun_out/r04b bash tools/gpu.sh "tests" "bench c2 --steps 20 --warmup 5" "trace c2 --steps 20 --warmup 5 --cpu-baseline-moves 0" "launch c2 --steps 20 --warmup 5 --cpu-baseline-moves 0" "bench c4 $C4" "trace c4 $C4" "bench c5 $C5" "trace c5 $C5"
