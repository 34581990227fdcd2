import torch
for dev in ['cpu', 'cuda']:
    x = torch.zeros(3, 1001, device=dev)
    x[:, 500] = 1.0; x[:, 1000] = 1.0; x[:, 7] = 1.0
    x[1, :] = torch.randn(1001, generator=torch.Generator().manual_seed(0)).to(dev)
    x[1, 990] = x[1].max() + 1; x[1, 3] = x[1, 990]
    v, i = torch.topk(x, 10)
    print(dev, i[0, :4].tolist(), i[1, :3].tolist())
    y = torch.flip(x, dims=[-1]); v, i = torch.topk(y, 10)
    print(dev, 'flipped', i[0, :4].tolist(), i[1, :3].tolist())
