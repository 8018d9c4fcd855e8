import sys, torch
sys.path[:0]=['/root/repo','/root/repo/tests','/root/repo/aimnet-x2d_amd']
import test_gpu_parity as T
for args in [(17,5,3,"NT"),(64,64,32,"NT"),(64,64,32,"NN"),(64,64,32,"TN"),(100,70,50,"NT"),(9170,76,76,"NT")]:
    C,col,pre,ref,_=T._gemm(*args, bias=False, res=False)
    d=(C.double()-ref).abs()
    print(args, 'maxerr', d.max().item(), 'refmax', ref.abs().max().item())
    if d.max().item()>1e-3:
        bad=(d>1e-3).nonzero()
        print('  bad count', bad.shape[0], 'first', bad[:5].tolist())
        print('  C[0,:4]', C[0,:4].tolist(), 'ref', ref[0,:4].tolist())
