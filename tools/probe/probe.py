import ctypes, os, sys, torch
lib = ctypes.CDLL(os.path.join(os.path.dirname(os.path.abspath(__file__)), 'libprobe.so'))
dev = torch.device('cuda:0')
s = torch.cuda.current_stream().cuda_stream
torch.manual_seed(0)
A = torch.randint(-4, 5, (32, 2)).float().to(dev); B = torch.randint(-4, 5, (2, 32)).float().to(dev)
C = torch.zeros(32, 32, device=dev)
r = lib.probe32(ctypes.c_void_p(A.data_ptr()), ctypes.c_void_p(B.data_ptr()), ctypes.c_void_p(C.data_ptr()), ctypes.c_void_p(s))
torch.cuda.synchronize()
print('rc', r, '32x32x2 maxerr', (C - A @ B).abs().max().item())
A = torch.randint(-4, 5, (16, 4)).float().to(dev); B = torch.randint(-4, 5, (4, 16)).float().to(dev)
C = torch.zeros(16, 16, device=dev)
r = lib.probe16(ctypes.c_void_p(A.data_ptr()), ctypes.c_void_p(B.data_ptr()), ctypes.c_void_p(C.data_ptr()), ctypes.c_void_p(s))
torch.cuda.synchronize()
print('rc', r, '16x16x4 maxerr', (C - A @ B).abs().max().item())
print(torch.cuda.get_device_name(0), torch.cuda.get_device_properties(0))
import subprocess
print(subprocess.run(['nproc'], capture_output=True, text=True).stdout, os.sched_getaffinity(0).__len__())
