import sys, os, numpy as np, torch
sys.path.insert(0, os.getcwd()); sys.path.insert(0, os.path.join(os.getcwd(), 'tests'))
from test_gpu_bitsliced import _wman
from oracle.philox_oracle import awgn_llr
dev = torch.device('cuda:0')
dec, cp = _wman(dev, sharing=(2, 0, 2), q=5, T=12)
s = float(cp.sigma(2.25))
llr = dec.awgn(9000, s, seed=11)
ref, _ = awgn_llr(9000, 576, s, 11, 0, decoding_type=2, q_bit=5)
g = llr.cpu().numpy()
print('sigma', s, 'channel equal', np.array_equal(g, ref), 'mismatches', int((g != ref).sum()), 'gpu mean', g.mean(), 'ref mean', ref.mean())
for k in ('flood', 'fused'):
    r = dec.decode(llr, app=False, counters=True, flags=True, kernel=k)
    print(k, r.counters.cpu().numpy(), dec.last_kernel())
r = dec.decode(torch.from_numpy(ref).to(dev), app=True)
app = r.app.cpu().numpy()
print('app>=0 frames', int((app >= 0).any(1).sum()))
