import sys, numpy as np
sys.path.insert(0, 'lz77-sss_amd'); sys.path.insert(0,'tests')
import lz77sss as lz
from conftest import load_golden
g = load_golden('zeros_10k'); T = g['text']
with lz.Session(1 << 22) as s:
    s.load(T); z = s.factorize(phr_mode=3); print(s.factors(z)[:5], flush=True)
