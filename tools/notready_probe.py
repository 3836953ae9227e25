"""Does hipEventQuery's hipErrorNotReady become HIP's last error (which torch's launch checks would
then report)?  Dev probe, under gpurun."""
import ctypes as C

import torch

hip = C.CDLL("libamdhip64.so")
torch.cuda.init()
s = torch.cuda.Stream()
with torch.cuda.stream(s):
    torch.cuda._sleep(200_000_000)
    e = torch.cuda.Event()
    e.record(s)
print("peek before", hip.hipPeekAtLastError())
q = hip.hipEventQuery(C.c_void_p(e.cuda_event))
print("query", q, "peek after", hip.hipPeekAtLastError())
x = torch.ones(4, device="cuda") * 2   # a torch kernel launch and its check
torch.cuda.synchronize()
print("torch op ok", float(x.sum()), "peek end", hip.hipPeekAtLastError())
