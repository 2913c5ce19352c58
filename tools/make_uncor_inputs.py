#!/usr/bin/env python3
"""Regenerate the post-decoder inputs the reference snapshot lacks (.MISSING_LARGE_BLOBS:1-3):
Inputs/[Uncor]_wman_N0576_R34_z24{,_Valid,_Test}.txt, i.e. the reference's sampling_type=2
collection (main_Base.py config: wman, sharing [3,0,3], QMS q=5, T=20, trained weights
Weights/C0_wman_N0576_R34_z24_Opt_Weight_End20.txt) run as a GPU sweep
(ldpc_error_floor_amd.fer.collect_uncor_inputs).  main_Post.py then reads them unchanged
(training_num 10000, valid_num 5000, test_num 5000 are the defaults here).

usage: python3 tools/make_uncor_inputs.py [--snr 3.0] [--out Inputs] [--counts 10000 5000 5000]
The reference fixes no collection SNR (check_params only requires a single one); 3.0 dB is
where its base decoder's FER is ~8e-2 (the SURVEY §8 c anchor)."""
import argparse
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
DATA = os.path.join(ROOT, "ldpc_error_floor_amd", "data")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--snr", type=float, default=3.0)
    ap.add_argument("--out", default="Inputs")
    ap.add_argument("--counts", type=int, nargs=3, default=[10000, 5000, 5000])
    ap.add_argument("--seed", type=int, default=1076)
    ap.add_argument("--batch", type=int, default=1 << 16)
    a = ap.parse_args()
    from ldpc_error_floor_amd.code import CodeParams
    from ldpc_error_floor_amd.decoder import Decoder
    name = "wman_N0576_R34_z24"
    dec = Decoder(os.path.join(DATA, "BaseGraph", name + ".txt"), 24, sharing=(3, 0, 3),
                  decoding_type=2, q_bit=5,
                  weights_txt=os.path.join(DATA, "Weights", f"C0_{name}_Opt_Weight_End20.txt"),
                  T=20, B_max=a.batch)
    sigma = float(CodeParams(dec.graph.proto, 24).sigma(a.snr))
    t0 = time.time()
    from ldpc_error_floor_amd.fer import collect_uncor_inputs
    res = collect_uncor_inputs(dec, sigma, name, a.counts, a.out, batch=a.batch, seed=a.seed)
    for path, (rows, decoded) in res.items():
        print(f"{path}: {rows} uncorrected words from {decoded} codewords at {a.snr} dB")
    print(f"done in {time.time() - t0:.1f} s")


if __name__ == "__main__":
    main()
