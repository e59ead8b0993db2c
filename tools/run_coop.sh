# long-path worker sweep (tuning): bench lines under gpurun_out/coop/
mkdir -p gpurun_out/coop
i=0
for a in "" "--long 64,64" "--long 128,512" "--long 48,256" "--long 96,1024" "--long 160,2048"; do
  i=$((i+1))
  SURF_DEBUG_TAIL=1 timeout -k 10 200 python bench.py --no-cpu --profile-pass 0 $a > gpurun_out/coop/r$i.json 2> gpurun_out/coop/r$i.err || exit 1
done
