import sys, time, os
sys.path.insert(0, os.environ.get('GRAFT_REPO_ROOT', '/root/repo'))
import numpy as np, torch, spartan_amd
from spartan_amd import expr, workloads
spartan_amd.initialize()
n = int(sys.argv[1]) if len(sys.argv) > 1 else 4000000
X = expr.rand(n, 128, dtype=np.float32, seed=21).force()
workloads.kmeans_fit(X, 256, 1)
torch.cuda.synchronize()
t = time.perf_counter(); workloads.kmeans_fit(X, 256, 2); torch.cuda.synchronize()
print('ms/iter', (time.perf_counter()-t)/2*1e3)
