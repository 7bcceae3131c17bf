"""Per-launch time of step kernels (cfdj_vm_kernel_bench ids in $KB_IDS, default 1-6) for each
libcfdj variant given on the command line (built by tools/build_variant.sh); one process
per variant.  python tools/variant_ab.py build/a/libcfdj.so build/b/libcfdj.so ..."""
import json, os, subprocess, sys

CODE = r'''
import math, os, sys, json
sys.path.insert(0, os.getcwd())
import numpy as np
from cfd_julia_amd import VortexMerger
from cfd_julia_amd.common import vm_ic
n = 4096; dx = 2 * math.pi / n
h = VortexMerger(n, n, dx, dx, 1000.0, device=0)
x = dx * np.arange(n + 1)
wn = np.zeros((n + 2, n + 2), order="F"); vm_ic(n, n, x, x, wn); h.upload(wn)
h.step(5e-4, 1)
print(json.dumps({k: round(h.kernel_bench(k, 5e-4, 20) * 1e3, 1) for k in [int(i) for i in os.environ.get("KB_IDS", "1,2,3,4,5,6").split(",")]}))
'''
for lib in sys.argv[1:]:
    env = dict(os.environ, CFDJ_LIB=lib)
    r = subprocess.run([sys.executable, "-c", CODE], env=env, capture_output=True, text=True,
                       timeout=120)
    print(lib, r.stdout.strip() or r.stderr.strip()[-400:], flush=True)
