import sys, numpy as np
sys.path.insert(0, '/root/repo')
import fractencode_amd as F
p = np.fromfile('/root/repo/tests/golden/crop64.u8', np.uint8).reshape(64, 64)
eng = int(sys.argv[1])
with F.Engine(0, 4, False, 0.0, -1.0, eng) as e:
    e.set_frame(p); e.set_domains(F.create_uniform_grid(64, 64, 16, 8))
    out, st = e.search(F.create_uniform_grid(64, 64, 8, 8))
print("engine", eng, "ok", st["engine"])
import torch
print("torch avail", torch.cuda.is_available(), torch.cuda.device_count())
torch.zeros(1).cuda()
print("torch ok")
