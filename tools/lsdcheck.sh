export LZ77SSS_LSD_CHECK=1 LZ77SSS_NO_PRED=1
python3 tools/rle_probe.py 1 7 2>&1 | grep -a "lsd-check\|  \[" | head -20
python3 tools/rle_probe.py 1024 42 2>&1 | grep -a "lsd-check\|  \[" | head -20
