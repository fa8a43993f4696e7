"""Time hipFFT (through torch.fft) variants for the 8192^2 dirty-image FFT."""
import torch, time
dev = "cuda"
n = 8192
g = torch.randn(n, n, dtype=torch.complex128, device=dev)
h = torch.randn(n, n // 2 + 1, dtype=torch.complex128, device=dev)
def t(f, reps=5):
    f(); torch.cuda.synchronize()
    a = time.perf_counter()
    for _ in range(reps): f()
    torch.cuda.synchronize()
    return (time.perf_counter() - a) / reps * 1e3
print("c2c fft2 in-place-ish", t(lambda: torch.fft.fft2(g)))
print("c2r irfft2", t(lambda: torch.fft.irfft2(h, s=(n, n))))
print("c2c 1d rows", t(lambda: torch.fft.fft(g, dim=1)))
print("c2c 1d cols", t(lambda: torch.fft.fft(g, dim=0)))
print("c2r 1d rows", t(lambda: torch.fft.irfft(h, n=n, dim=1)))
hc = h[:, :].contiguous()
print("c2c 1d cols on half", t(lambda: torch.fft.fft(hc, dim=0)))
