set -e
bash tools/_lat8b.sh
timeout -k 10 400 python -u tools/tp8_rank_emulation.py --md gpurun_out/tp8_proj.md > gpurun_out/tp8.json 2> gpurun_out/tp8.err
