"""HBM write/copy rates for the block's activation sizes (reference points for the GEMM epilogues)."""
import torch


def tm(fn, it=20):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(it):
        fn()
    e1.record()
    e1.synchronize()
    return e0.elapsed_time(e1) / it * 1e3


for mb in (24.6, 49.2, 98.3, 196.6):
    n = int(mb * 1e6 / 2)
    x = torch.empty(n, dtype=torch.bfloat16, device="cuda")
    y = torch.empty(n, dtype=torch.bfloat16, device="cuda")
    t_fill = tm(lambda: x.fill_(1.0))
    t_copy = tm(lambda: y.copy_(x))
    print(f"{mb:6.1f} MB: fill {t_fill:7.1f} us ({mb*1e-3/t_fill*1e3:5.2f} TB/s)  copy {t_copy:7.1f} us "
          f"({2*mb*1e-3/t_copy*1e3:5.2f} TB/s r+w)", flush=True)
