import ctypes as C, sys
sys.path.insert(0,'skyvault-rs_amd')
import torch; torch.cuda.init()
from skv import gen
from skv.api import Compactor
c=Compactor(0)
for k in (6,96,200):
    s=gen.config2(seed=1,n_streams=k,n_records=400,vsize=40,variant="B")
    r=c.compact(s,64<<10,0); print(k,len(r),c.timings()["path"])
