# drain segment anatomy on the current tree + the 8-shard C3 projection
mkdir -p gpurun_out/r4/seg
timeout -k 10 200 python tools/segment_cycles.py 48 > gpurun_out/r4/seg/segment_cycles.json 2> gpurun_out/r4/seg/segment_cycles.err || exit 2
cat gpurun_out/r4/seg/segment_cycles.json
timeout -k 10 600 python tools/shard_probe.py 8 > gpurun_out/r4/seg/shards8_c3.txt 2> gpurun_out/r4/seg/shards8_c3.err || exit 3
tail -1 gpurun_out/r4/seg/shards8_c3.txt
