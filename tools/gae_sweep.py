"""Micro-sweep of the GAE prefetch depth at the §8d shape (diagnostic)."""
import os, subprocess, sys, json
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
code = r'''
import sys, torch, numpy as np
sys.path.insert(0, "%s")
from agilerl_amd import kernels as K
P,T,N=8,1024,8192
g=torch.Generator(device="cuda").manual_seed(0)
r=torch.randn(P,T,N,device="cuda",generator=g); v=torch.randn_like(r)
d=(torch.rand(P,T,N,device="cuda",generator=g)<0.01).to(torch.uint8)
lv=torch.randn(P,N,device="cuda"); ld=torch.zeros(P,N,dtype=torch.uint8,device="cuda")
adv=torch.empty_like(r); ret=torch.empty_like(r)
for _ in range(3): K.gae(r,d,v,lv,ld,advantages=adv,returns=ret)
torch.cuda.synchronize()
s=torch.cuda.Event(enable_timing=True); e=torch.cuda.Event(enable_timing=True)
s.record()
for _ in range(10): K.gae(r,d,v,lv,ld,advantages=adv,returns=ret)
e.record(); e.synchronize(); ms=s.elapsed_time(e)/10
print(ms, 17*P*T*N/ms/1e6)
''' % ROOT
for u in sys.argv[1:] or ["8", "16", "32"]:
    env = dict(os.environ, AGX_GAE_UNROLL=u)
    out = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True)
    print("U=", u, out.stdout.strip(), out.stderr.strip()[-300:])
