"""The roofline pair alone at S scans per launch (bench.py's roofline_at), for a rocprofv3 PMC pass whose
per-dispatch figures then match bench.py's `roofline.at_roofline_streams` (tools/pmc_summarize.py
--streams S).  python tools/roofline_pmc.py [S] [vlp16|hdl64]"""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "lego-loam-bor_amd"))


def main():
    import torch
    import bench
    import lego_amd as L
    from lego_amd import _abi as A
    S = int(sys.argv[1]) if len(sys.argv) > 1 else 2048
    kind = sys.argv[2] if len(sys.argv) > 2 else "vlp16"
    sys.argv = [sys.argv[0], "--roofline-streams", str(S), "--roofline-reps", "3", "--kind", kind]
    args = bench.parse()
    cfg = A.synth_cfg(args.kind)
    stream = torch.cuda.Stream()
    mk_params = L.params_vlp16 if args.kind == "vlp16" else L.params_hdl64
    print(bench.roofline_at(args, L, A, mk_params, cfg, 0, stream))


if __name__ == "__main__":
    main()
