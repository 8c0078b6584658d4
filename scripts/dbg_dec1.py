"""Debug: compare dec1 backward buffers (dout, dy2, dy1) with the fp64 oracle."""
import sys; sys.path[:0]=['tests','.','spff-unet-spcct_amd']
import numpy as np, torch, torch.nn.functional as F
from _golden import load, cfg_of, state_of
from oracle import spff_oracle as O
import test_gpu_parity as T
import innovative3D.helpers as Hh
from innovative3D import _engine as E
name = sys.argv[1] if len(sys.argv) > 1 else "fx1b_config1_k9"
d=load(name); cfg=cfg_of(d["meta"]); st=state_of(d); K=d["meta"]["K"]
P=O.params_from_state(st, dtype=torch.float64)
x=torch.from_numpy(d["x"]).double(); y=torch.from_numpy(d["labels"])
cap={}
def hooked(P_,pre,inp,ksd):
    w=P_[pre+".0.weight"]
    yv=F.conv3d(inp,w,None,padding=(ksd//2,1,1)); yv.retain_grad(); cap[pre]=yv
    return F.leaky_relu(F.instance_norm(yv,weight=P_[pre+".1.weight"],bias=P_[pre+".1.bias"],eps=1e-5),0.01)
O.conv_in_lrelu=hooked
orig_nb=O.novel_block
def nb(P_,pre,inp,cfg_):
    o=orig_nb(P_,pre,inp,cfg_); o.retain_grad(); cap[pre+".out"]=o; return o
O.novel_block=nb
O.fwd_bwd(P,x,y,cfg)
core=T.load_core(d)
xx=torch.from_numpy(d["x"]).cuda(); yy=torch.from_numpy(d["labels"]).cuda()
logits=core(xx); loss,conf=Hh.ce_dice_with_confusion(logits,yy,K,255)
plan=core._plan
E.check(E.lib().spff_debug_set(plan._h,0,1),"dbg")
loss.backward(); torch.cuda.synchronize()
def cl(t): return t.permute(0,2,3,4,1).reshape(-1,t.shape[1]).numpy()
def cmp(tag, mine, ref):
    e=np.abs(mine-ref).max()/max(np.abs(ref).max(),1e-30); print(f"  {tag:10s} rel {e:.3e}  (absmax ref {np.abs(ref).max():.3e})")
V=d["x"].shape[0]*d["x"].shape[2]*d["x"].shape[3]*d["x"].shape[4]; C=cfg.base
g=lambda n: plan.saved(n).cpu().numpy()[:V,:C]
cmp("dout", g("grad.out"), cl(cap["dec1.out"].grad))
cmp("dy2", g("grad.dy2"), cl(cap["dec1.body"].grad))
cmp("dy1", g("grad.da1"), cl(cap["dec1.pre"].grad))
np.savez_compressed(f"gpurun_out/dbg_{name}.npz", dout=g("grad.out"), dout_ref=cl(cap["dec1.out"].grad),
                    dy2=g("grad.dy2"), dy2_ref=cl(cap["dec1.body"].grad),
                    y2=plan.saved("dec1.y2").cpu().numpy(), y2_ref=cl(cap["dec1.body"].detach()))
