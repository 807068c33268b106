set -e
timeout -k 10 300 python -u tools/c2_probe.py --digest > gpurun_out/c2_probe_d.json 2> gpurun_out/c2_probe_d.err
timeout -k 10 300 python -u tools/c2_probe.py > gpurun_out/c2_probe.json 2> gpurun_out/c2_probe.err
echo done
