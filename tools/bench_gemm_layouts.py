import json, torch, sys
import os; sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from tools.bench_gemms import timeit
T=16384; bf=torch.bfloat16
for name,(K,N) in {"qkv":(4096,6144),"o":(4096,4096),"gu":(4096,28672),"down":(14336,4096),"lm":(4096,128256)}.items():
    aug = 0 if name=="lm" else 64
    dy = torch.randn(T, N+aug, device="cuda", dtype=bf)
    W2 = torch.randn(N+aug, K, device="cuda", dtype=bf)
    W2T = W2.t().contiguous()
    nn = timeit(lambda: dy @ W2)
    tn = timeit(lambda: dy @ W2T.t())
    fl = 2*T*N*K
    print(json.dumps({"gemm":name,"nn_ms":round(nn,3),"nn_tf":round(fl/nn/1e9),"tn_ms":round(tn,3),"tn_tf":round(fl/tn/1e9)}), flush=True)
