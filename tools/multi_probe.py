"""Debug probe: a multi-device handle as the process's first HIP use (AMD_LOG_LEVEL shows
failing HIP calls)."""
import sys, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import pkgload
pkg = pkgload.load()
b, o = pkg.keys.pack(["k%d" % i for i in range(1000)])
print("multi", flush=True)
with pkg.Filter(9585058, 6, devices=[0], mode="replicated") as f:
    print("created", flush=True)
    f.insert_many(b, o)
print("ok", flush=True)
