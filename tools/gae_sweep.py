"""Micro-sweep of the GAE kernel at the §8d shape (diagnostic):
prefetch depth (AGX_GAE_UNROLL) x columns per lane (AGX_GAE_COLS), with and
without the fused advantage statistics."""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
code = r'''
import sys, torch
sys.path.insert(0, "%s")
from agilerl_amd import kernels as K
P,T,N=8,1024,8192
g=torch.Generator(device="cuda").manual_seed(0)
r=torch.randn(P,T,N,device="cuda",generator=g); v=torch.randn_like(r)
d=(torch.rand(P,T,N,device="cuda",generator=g)<0.01).to(torch.uint8)
lv=torch.randn(P,N,device="cuda"); ld=torch.zeros(P,N,dtype=torch.uint8,device="cuda")
adv=torch.empty_like(r); ret=torch.empty_like(r)
st=torch.empty(P,2,dtype=torch.float64,device="cuda")
for stats in (False, True):
    run=lambda: K.gae(r,d,v,lv,ld,advantages=adv,returns=ret,with_stats=stats,stats_out=st if stats else None)
    for _ in range(3): run()
    torch.cuda.synchronize()
    s=torch.cuda.Event(enable_timing=True); e=torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(10): run()
    e.record(); e.synchronize(); ms=s.elapsed_time(e)/10
    print("stats" if stats else "plain", round(ms, 4), "ms", round(17*P*T*N/ms/1e6, 1), "GB/s")
''' % ROOT
for cols in (sys.argv[1].split(",") if len(sys.argv) > 1 else ["1", "2"]):
    for u in (sys.argv[2].split(",") if len(sys.argv) > 2 else ["8", "16", "32"]):
        env = dict(os.environ, AGX_GAE_UNROLL=u, AGX_GAE_COLS=cols)
        out = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True)
        print(f"cols={cols} U={u}:", out.stdout.strip().replace("\n", " | "), out.stderr.strip()[-300:])
