import torch, sys
sys.path.insert(0, "buck-gnn_amd")
dev = torch.device("cuda", 0)
torch.manual_seed(0)
for (m, k, n) in [(1024, 512, 128), (1024, 128, 512), (512, 1024, 128)]:
    a = torch.randn(m, k, device=dev) * 0.05
    b = torch.randn(k, n, device=dev) * 0.05
    c = torch.mm(a, b)
    r = a.double() @ b.double()
    mag = a.abs().double() @ b.abs().double()
    print(m, k, n, "torch.mm max rel-to-|A||B| err", ((c.double() - r).abs() / mag).max().item(),
          "allow_tf32", torch.backends.cuda.matmul.allow_tf32, torch.get_float32_matmul_precision())
