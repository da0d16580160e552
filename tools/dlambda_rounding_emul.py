"""CPU emulation (fp64 with selective bf16 roundings) of which rounding dominates the d(coef) error
of one diff-attention layer whose dO is LayerNorm-projected, as in the default-config model (the
cancellation that makes d(lambda) ill-conditioned).  Round-6 evidence for DESIGN "bf16 d(lambda)";
output in profiles/r06_dlambda_rounding_emul.txt.   python tools/dlambda_rounding_emul.py"""
# CPU emulation: which rounding dominates d(coef) error for one diff-attention layer whose dO is
# LayerNorm-projected (the cancellation of the default-config model).  fp64 baseline.
import torch, math
torch.manual_seed(0)
B,T,H,hs = 2,512,4,96
dv = 2*hs
def bf(x): return x.to(torch.bfloat16).double()
q = [torch.randn(B,H,T,hs,dtype=torch.float64)*0.5 for _ in range(2)]
k = [torch.randn(B,H,T,hs,dtype=torch.float64)*0.5 for _ in range(2)]
v = torch.randn(B,H,T,dv,dtype=torch.float64)
q=[bf(x) for x in q]; k=[bf(x) for x in k]; v=bf(v)      # bf16 activations on both sides
lam = 0.47
mask = torch.ones(T,T,dtype=torch.bool).tril()
def probs(qi,ki,round_scores=False):
    s = qi@ki.transpose(-1,-2)/math.sqrt(hs)
    if round_scores: s = bf(s)
    s = s.masked_fill(~mask, float('-inf'))
    return torch.softmax(s,-1)
A = [probs(q[i],k[i]) for i in range(2)]
O_i = [a@v for a in A]
O = O_i[0] - lam*O_i[1]                       # (B,H,T,dv)
# LN backward projection across heads: dX ⊥ (X - mean) and ⊥ 1 per token
X = O.permute(0,2,1,3).reshape(B,T,H*dv)
g = torch.randn(B,T,H*dv,dtype=torch.float64)
xc = X - X.mean(-1,keepdim=True)
def proj(d):
    d = d - d.mean(-1,keepdim=True)
    return d - (d*xc).sum(-1,keepdim=True)/(xc*xc).sum(-1,keepdim=True)*xc
dX = proj(g)
dO = dX.reshape(B,T,H,dv).permute(0,2,1,3)
def dcoef(dOx, Oix): return torch.stack([(dOx*o).sum(dim=(0,2,3)) for o in Oix],-1)   # (H, 2)
exact = dcoef(dO, O_i)
def err(x): return ((x-exact).abs()/exact.abs()).max(0).values   # per branch, max over heads
print('exact dcoef', exact)
print('terms scale', torch.stack([(dO*o).abs().sum(dim=(0,2,3)) for o in O_i],-1))
# ours: dO rounded to bf16; O_i from bf16-rounded P (fp32 accumulate ~ exact here)
print('ours: bf16 dO only        ', err(dcoef(bf(dO), O_i)))
print('ours: bf16 P in O_i only  ', err(dcoef(dO, [bf(a)@v for a in A])))
print('ours: both                ', err(dcoef(bf(dO), [bf(a)@v for a in A])))
# reference under autocast: scores rounded to bf16, grad_diff = bf16(dO @ v^T), dlam from fp32 A2
Ar = [probs(q[i],k[i],True) for i in range(2)]
gd = bf(bf(dO)@v.transpose(-1,-2))
ref = torch.stack([(gd*a).sum(dim=(0,2,3)) for a in Ar],-1)
print('ref route: bf16 scores + bf16 grad_diff', err(ref))
gd0 = bf(dO)@v.transpose(-1,-2)
print('ref route: bf16 dO only   ', err(torch.stack([(gd0*a).sum(dim=(0,2,3)) for a in A],-1)))
print('ref route: bf16 scores only', err(torch.stack([((dO@v.transpose(-1,-2))*a).sum(dim=(0,2,3)) for a in Ar],-1)))
