import sys; sys.path[:0]=['tests','.','spff-unet-spcct_amd']
import numpy as np, torch
from _golden import load, cfg_of, state_of
import test_gpu_parity as T
import innovative3D.helpers as Hh
for name in sys.argv[1:]:
    d=load(name); K=d["meta"]["K"]
    core=T.load_core(d)
    x=torch.from_numpy(d["x"]).cuda(); y=torch.from_numpy(d["labels"]).cuda()
    loss,conf=Hh.ce_dice_with_confusion(core(x),y,K,255); loss.backward(); torch.cuda.synchronize()
    r64,r32=T.oracle_grads(d)
    named=dict(core.named_parameters(remove_duplicate=False))
    print("==",name)
    for kk,g64 in r64.items():
        g=named[kk].grad.double().cpu().numpy(); s=max(np.abs(g64).max(),1e-12)
        e=np.abs(g-g64).max()/s; e32=np.abs(r32[kk]-g64).max()/s
        flag = "  <<<" if e > max(1e-3, 8*e32) else ""
        print(f"  {kk:32s} {e:.2e} {e32:.2e}{flag}")
