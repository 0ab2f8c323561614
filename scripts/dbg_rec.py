# debug: decode selected golden records alone and report mismatching elements
import sys, numpy as np
sys.path.insert(0, 'tests'); sys.path.insert(0, 'turbopfor-cpp_amd/python')
import torch, golden_io, turbopfor_amd as tpf
recs = [r for r in golden_io.load('g256v32.bin') if r.n == 256 and not r.d1]
for i in [int(x) for x in sys.argv[1:]]:
    r = recs[i]
    packed = torch.from_numpy(np.frombuffer(r.enc, dtype=np.uint8).copy()).cuda()
    offs = torch.tensor([0, len(r.enc)], dtype=torch.int64, device='cuda')
    err = torch.full((1,), -1, dtype=torch.int64, device='cuda')
    out = tpf.dec256v32(packed, offs, 1, err=err)
    got = out.cpu().numpy().view(np.uint32).reshape(-1)
    bad = np.nonzero(got != r.values)[0]
    print(i, 'err', err.item(), 'nbad', len(bad), bad[:16].tolist(), [hex(int(got[j])) for j in bad[:6]], [hex(int(r.values[j])) for j in bad[:6]])
