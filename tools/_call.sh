bash tools/gpu.sh tests && bash tools/gpu.sh bench --steps 20 --warmup 5 && \
bash tools/gpu.sh rehearsal 2 4 && \
timeout -k 10 200 python tools/plane_probe.py --P 8 --sizes 16M 256M --rounds 30 --stamps > gpurun_out/probe_p8.jsonl 2> gpurun_out/probe_p8.err && \
timeout -k 10 200 python tools/plane_probe.py --P 2 --sizes 256M --units 256 --rounds 30 > gpurun_out/probe_split.jsonl 2>> gpurun_out/probe_split.err && \
timeout -k 10 200 python tools/plane_probe.py --P 2 --sizes 256M --units 4 --rounds 30 >> gpurun_out/probe_split.jsonl 2>> gpurun_out/probe_split.err && \
timeout -k 10 200 python tools/plane_probe.py --P 2 --sizes 1M 40 --rounds 200 --stamps > gpurun_out/probe_small_stamps.jsonl 2>> gpurun_out/probe_split.err
