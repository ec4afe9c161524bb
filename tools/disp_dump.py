import sys, torch, numpy as np
from leastereo_amd import kernels
g = torch.Generator().manual_seed(3)
outs = []
for shape, md in [((1, 1, 64, 192, 320), 192), ((2, 1, 32, 17, 29), 96), ((1, 1, 64, 12, 20), 192)]:
    x = (torch.randn(shape, generator=g) * float(sys.argv[2])).cuda()
    y = kernels.disparity_regression(x, md)
    torch.cuda.synchronize()
    outs.append(y.cpu().numpy().ravel())
    if shape[2] == 64 and shape[3] == 192:
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
        for _ in range(3): kernels.disparity_regression(x, md)
        ev[0].record()
        for _ in range(20): kernels.disparity_regression(x, md)
        ev[1].record(); torch.cuda.synchronize()
        print(sys.argv[1], "C2 disparity us", ev[0].elapsed_time(ev[1]) / 20 * 1e3)
np.save(sys.argv[1], np.concatenate(outs))
