import ctypes, os, sys, torch
here = os.path.dirname(os.path.abspath(__file__))
lib = ctypes.CDLL(os.path.join(here, "probe_dpp.so"))
x = torch.arange(64, dtype=torch.float32, device="cuda")
out = torch.zeros(9 * 64, dtype=torch.float32, device="cuda")
rc = lib.probe_launch(ctypes.c_void_p(x.data_ptr()), ctypes.c_void_p(out.data_ptr()),
                      ctypes.c_void_p(torch.cuda.current_stream().cuda_stream))
torch.cuda.synchronize()
print("rc", rc)
names = ["row_ror1", "row_ror15", "row_newbcast3", "row_shr1", "pl32swap0", "pl32swap1", "pl16swap0", "pl16swap1", "fmac_dpp_ror3"]
o = out.view(9, 64).cpu()
for i, n in enumerate(names):
    print(n, o[i].int().tolist())
