import time, torch
torch.zeros(1, device="cuda")
dev = torch.device("cuda", 0)
def t(f, n=20000):
    f()
    t0 = time.perf_counter()
    for _ in range(n): f()
    return (time.perf_counter() - t0) / n * 1e6
print("current_stream().cuda_stream", t(lambda: torch.cuda.current_stream().cuda_stream))
print("current_stream(dev).cuda_stream", t(lambda: torch.cuda.current_stream(dev).cuda_stream))
print("_cuda_getCurrentRawStream(0)", t(lambda: torch._C._cuda_getCurrentRawStream(0)))
print("current_device()", t(lambda: torch.cuda.current_device()))
print("_cuda_getDevice()", t(lambda: torch._C._cuda_getDevice()))
x = torch.zeros(10, device="cuda")
print("data_ptr", t(lambda: x.data_ptr()))
e = torch.cuda.Event()
print("Event.record", t(lambda: e.record()))
with torch.cuda.stream(torch.cuda.Stream()):
    print("in side stream raw", torch._C._cuda_getCurrentRawStream(0) == torch.cuda.current_stream().cuda_stream)
