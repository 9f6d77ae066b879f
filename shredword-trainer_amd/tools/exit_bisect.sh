# Diagnostic: which library loaded before torch makes `import torch` + a CUDA op abort at exit.
export LD_LIBRARY_PATH=/opt/rocm/lib
run() {
  timeout -k 5 120 python -c "
import ctypes
for n in '$1'.split(','):
    if n: ctypes.CDLL(n, mode=ctypes.RTLD_GLOBAL)
import torch
print(torch.ones(3, device='cuda').sum().item())" > /dev/null 2>&1
  echo "$1 rc=$?"
}
run libamdhip64.so,librccl.so
run libamdhip64.so,libroctx64.so
run libamdhip64.so,libnuma.so
run libamdhip64.so,libamd_comgr.so
run libamdhip64.so,librocprofiler-register.so,libhsa-runtime64.so
run shredword-trainer_amd/shredword/libtrainer.so
run libamdhip64.so,libhsa-runtime64.so,librocprofiler-register.so,libamd_comgr.so,librccl.so,libroctx64.so,libnuma.so
