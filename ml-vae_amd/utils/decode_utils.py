"""MD-VAE decoding on libmlvae (replaces ref:src/utils/decode_utils.py).

``decode_plvl_md_lbl_seqs_full`` -- the Viterbi decode the MD-VAE training forward runs
(ref:src/models/MD_VAE/model.py:20,133-141; ref:src/utils/decode_utils.py:374-565) -- runs as one
kernel over the batch (csrc/decode.hip, one workgroup per utterance) instead of a joblib pool of
host DPs.  Same arguments and return value: lists (per utterance) of the decoded boundary
sequence (np.ndarray of 0/1), the frame-level and the phoneme-level mispronunciation labels.
The reference's backtrack assertion raises AssertionError likewise.  ``decode_plvl_md_lbl_seqs``
is the name the MD-VAE model imports it under.
"""
import numpy as np
import torch

from mlvae_hip._lib import check, lib


def _f32(t, dev):
    return t.to(dev, torch.float32).contiguous()


def decode_plvl_md_lbl_seqs_full(predictions, utt_ids, feat_lens, plvl_cnnl_seqs, plvl_cnnl_seq_lens,
                                 prior, weight=1.0):
    logits = predictions["phn_recog_out"]
    if not logits.is_cuda:
        raise RuntimeError("decode_plvl_md_lbl_seqs_full runs on the HIP device only (no CPU fallback)")
    dev = logits.device
    logits = _f32(logits, dev)
    B, T, N = logits.shape
    L = plvl_cnnl_seqs.shape[1]
    bv = _f32(predictions["boundary_v"], dev)
    pil = _f32(predictions["pi_logits"], dev)
    seqs = plvl_cnnl_seqs.to(dev, torch.int64).contiguous()
    fl, sl, pr = _f32(feat_lens, dev), _f32(plvl_cnnl_seq_lens, dev), _f32(prior, dev)
    ws = torch.empty(max(lib().mlvae_viterbi_workspace_size(B, T, L), 1), device=dev, dtype=torch.uint8)
    bnd = torch.empty(B, T, device=dev, dtype=torch.int32)
    flvl = torch.empty(B, T, device=dev, dtype=torch.int32)
    plvl = torch.empty(B, L, device=dev, dtype=torch.int32)
    lens = torch.empty(B, 2, device=dev, dtype=torch.int32)
    err = torch.zeros(1, device=dev, dtype=torch.int32)
    P = lambda t: t.data_ptr()
    check(lib().mlvae_viterbi_md(B, T, N, L, P(logits), N, P(bv), P(pil), P(pr), P(seqs), P(fl), P(sl),
                                 float(weight), P(ws), ws.numel(), P(bnd), P(flvl), P(plvl), P(lens),
                                 P(err), torch.cuda.current_stream(dev).cuda_stream), "viterbi_md")
    host = [t.cpu().numpy() for t in (bnd, flvl, plvl, lens, err)]  # the one host sync of the decode
    bnd, flvl, plvl, lens, code = host
    if int(code[0]):
        raise AssertionError(f"MD decode: backtrack did not end at (0, 0) / empty utterance (err {int(code[0])})")
    out_b, out_f, out_p = [], [], []
    for i in range(B):
        Ti, Li = int(lens[i, 0]), int(lens[i, 1])
        out_b.append(bnd[i, :Ti].astype(np.int64))
        out_f.append([int(v) for v in flvl[i, :Ti]])
        out_p.append([int(v) for v in plvl[i, :Li]])
    return out_b, out_f, out_p


decode_plvl_md_lbl_seqs = decode_plvl_md_lbl_seqs_full
