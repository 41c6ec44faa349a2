import os, sys, torch
sys.path[:0] = ["/root/repo", "/root/repo/vision-language-pretraining-for-bone-tumor-detection_amd"]
from vlp_amd import ops
dev = torch.device("cuda", 0)
M, D = 10240, 312
dy = torch.randn(M, D, device=dev).to(torch.bfloat16); x = torch.randn(M, D, device=dev).to(torch.bfloat16)
mean = torch.zeros(M, device=dev); rstd = torch.ones(M, device=dev); gamma = torch.ones(D, device=dev)
dx = torch.empty_like(dy); dxd = torch.empty_like(dy); dg = torch.zeros(D, device=dev); db = torch.zeros(D, device=dev)
ad = torch.randn_like(dy)
def f(): ops.layernorm_bwd(dy, x, mean, rstd, gamma, dx, dxd, dg, db, M, D, p_out=0.1, seed_out=3, p_in=0.1, seed_in=4)
def g(): ops.layernorm_bwd_add(dy, x, mean, rstd, gamma, ad, dx, dg, db, M, D)
for fn, nm in ((f, "ln_bwd drop"), (g, "ln_bwd_add")):
    for _ in range(3): fn()
    torch.cuda.synchronize(); e0 = torch.cuda.Event(enable_timing=True); e1 = torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(20): fn()
    e1.record(); torch.cuda.synchronize()
    print(nm, os.environ.get("VLP_LNB_BLOCKS"), round(e0.elapsed_time(e1) / 20 * 1000, 1), "us")
