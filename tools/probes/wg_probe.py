import torch, sys
sys.path.insert(0, '.')
from pytorch_cifar_amd import _native
C = _native.lib()
torch.manual_seed(0)
def run(N, H, Cin, Cout, k, s, p):
    x = torch.randn(N, Cin, H, H, device='cuda').bfloat16().float().requires_grad_(True)
    w = torch.randn(Cout, Cin, k, k, device='cuda').bfloat16().float().requires_grad_(True)
    y = torch.nn.functional.conv2d(x, w, stride=s, padding=p)
    dy = torch.randn_like(y).bfloat16().float()
    y.backward(dy)
    xn = x.detach().permute(0,2,3,1).contiguous().bfloat16()
    dyn = dy.permute(0,2,3,1).contiguous().bfloat16()
    dw = C.conv_wgrad(xn, dyn, k, k, s, p, 1, None).permute(0,3,1,2)
    ref = w.grad
    err = ((dw-ref).abs().max()/ref.abs().max()).item()
    print(N,H,Cin,Cout,k,s,p,'err',err)
    if err > 0.05:
        r2 = ref.reshape(Cout, -1); d2 = dw.reshape(Cout, -1)
        print(' ref[:2,:8]', r2[:2,:8].tolist()); print(' got[:2,:8]', d2[:2,:8].tolist())
        # try to find column permutation
        for i in range(min(4, d2.shape[1])):
            c = (r2 - d2[:, i:i+1]).abs().sum(0)
            print('  got col', i, 'best ref col', c.argmin().item(), c.min().item())
        for i in range(min(4, d2.shape[0])):
            c = (r2 - d2[i:i+1, :]).abs().sum(1)
            print('  got row', i, 'best ref row', c.argmin().item(), c.min().item())
run(1, 8, 8, 8, 1, 1, 0)
run(1, 8, 8, 32, 1, 1, 0)
run(1, 8, 64, 64, 1, 1, 0)
run(2, 8, 64, 64, 3, 1, 1)
run(1, 8, 128, 128, 1, 1, 0)
