timeout -k 10 300 python -u tools/txseg_host_probe.py > gpurun_out/r02bd.jsonl 2>&1
