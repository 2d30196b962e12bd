set -o pipefail
O=gpurun_out/fd6; mkdir -p $O
timeout -k 10 200 python -u tools/fill_drain.py --windows 2 --steps 640 --warmup 5 > $O/long.jsonl 2>$O/long.err &&
timeout -k 10 200 python -u tools/fill_drain.py --windows 5 --steps 20 --warmup 5 > $O/short.jsonl 2>$O/short.err &&
timeout -k 10 200 python -u tools/fill_drain.py --windows 5 --steps 20 --warmup 5 --events 0 > $O/short_noev.jsonl 2>$O/short_noev.err
