"""Probe, not product: timings of the dense ops around the MaxK aggregation in one
ogbn-products-sized SAGE epoch (N = 2.45M rows, hidden 256, 47 classes), to choose
the forms maxk_layers / maxk_train_bench use.  Prints one line per variant (ms)."""
import torch

torch.backends.cuda.matmul.allow_tf32 = False
dev = torch.device("cuda")
N, H, C = 2449029, 256, 47


def t(f, n=5):
    f()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(n):
        f()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / n


g = torch.randn(N, H, device=dev)
x = torch.randn(N, H, device=dev)
W = torch.randn(H, H, device=dev)
for lib in ("default", "cublas", "cublaslt"):
    if lib != "default":
        try:
            torch.backends.cuda.preferred_blas_library(lib)
        except Exception as exc:  # noqa: BLE001
            print(lib, "unavailable", exc)
            continue
    print(f"[{lib}] fwd x@W^T        {t(lambda: x @ W.t()):.3f}")
    print(f"[{lib}] dW g^T@x         {t(lambda: g.t() @ x):.3f}")
    print(f"[{lib}] dW (x^T@g)^T     {t(lambda: (x.t() @ g).t()):.3f}")
    print(f"[{lib}] dX g@W           {t(lambda: g @ W):.3f}")
    for c in (8, 32, 128):
        m = N // c * c

        def chunked(c=c, m=m):
            gb = g[:m].view(c, m // c, H)
            xb = x[:m].view(c, m // c, H)
            return torch.bmm(gb.transpose(1, 2), xb).sum(0) + g[m:].t() @ x[m:]
        print(f"[{lib}] dW chunked bmm {c:4d} {t(chunked):.3f}")
torch.backends.cuda.preferred_blas_library("default") if hasattr(torch.backends.cuda, "preferred_blas_library") else None

logits = torch.randn(N, C, device=dev, requires_grad=True)
y = torch.randint(0, C, (N,), device=dev)


def ce_torch():
    loss = torch.nn.functional.cross_entropy(logits, y)
    loss.backward()


def ce_gather():
    lp = torch.log_softmax(logits, 1)
    loss = -lp.gather(1, y[:, None]).mean()
    loss.backward()


print(f"cross_entropy fwd+bwd torch   {t(ce_torch):.3f}")
print(f"cross_entropy fwd+bwd gather  {t(ce_gather):.3f}")
gC = torch.randn(N, C, device=dev)
ones = torch.ones(N, device=dev)
print(f"bias grad [N,47] sum(0)       {t(lambda: gC.sum(0)):.3f}")
print(f"bias grad [N,47] ones@g       {t(lambda: ones @ gC):.3f}")
print(f"bias grad [N,47] t().sum(1)   {t(lambda: gC.t().contiguous().sum(1)):.3f}")
print(f"bias grad [N,256] sum(0)      {t(lambda: g.sum(0)):.3f}")
print(f"bias grad [N,256] ones@g      {t(lambda: ones @ g):.3f}")

# ---- second round: bias-gradient forms and chunk counts
for c in (64, 128, 256, 512):
    m = N // c * c

    def chunked(c=c, m=m):
        return torch.bmm(g[:m].view(c, m // c, H).transpose(1, 2), x[:m].view(c, m // c, H)).sum(0)
    print(f"dW chunked bmm {c:4d} (no tail) {t(chunked):.3f}")
for c in (64, 128, 512):
    m = N // c * c
    print(f"bias [N,47] view({c}).sum(1).sum(0)  {t(lambda: gC[:m].view(c, m // c, C).sum(1).sum(0)):.3f}")
    oc = torch.ones(c, 1, m // c, device=dev)
    print(f"bias [N,47] bmm ones ({c})           {t(lambda: torch.bmm(oc, gC[:m].view(c, m // c, C)).sum(0)):.3f}")
xs = torch.randn(N, C, device=dev)
Wc = torch.randn(C, H, device=dev)
print(f"lin_out fwd x@W^T [N,256]x[256,47]   {t(lambda: x @ Wc.t()):.3f}")
print(f"lin_out dX gC@Wc                     {t(lambda: gC @ Wc):.3f}")
print(f"lin_out dW gC^T@x                    {t(lambda: gC.t() @ x):.3f}")
m = N // 128 * 128
print(f"lin_out dW chunked 128               {t(lambda: torch.bmm(gC[:m].view(128, m // 128, C).transpose(1, 2), x[:m].view(128, m // 128, H)).sum(0)):.3f}")
b = torch.randn(H, device=dev)
x2 = torch.randn(N, H, device=dev)
print(f"two addmm + add                      {t(lambda: torch.addmm(b, x, W.t()) + x2 @ W.t()):.3f}")
print(f"addmm + addmm_ (beta=1 accumulate)   {t(lambda: torch.addmm(b, x, W.t()).addmm_(x2, W.t())):.3f}")
