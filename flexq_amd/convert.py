"""Offline weight converter and on-disk packed-weight format.

The reference's serving path loads pre-packed 6-bit weights per tensor-parallel rank
(`LlamaDecoderLayerWeight.cc:381-410`: `*.attention.query_key_value.weight.<rank>.bin`, ...), but
the converter that writes them is not in the repository.  This module is that converter for this
engine: fp16 HF weights -> per-(row, 128-group) symmetric 6-bit codes with the engine rounding
rule (fq_quantize_pack_w6, the same rule as the activation quantizer) -> the weight image (codes
in fq6 blocks + blocked fp16 scales) -> one `.fqw6` file per linear and rank.

File layout (little-endian, 64-byte header, then the image exactly as the GEMM reads it):
  0  magic  b"FQW6IMG\\0"           32 tp_rank  i32
  8  version u32 (1)                36 tp_size  i32
  12 header bytes u32 (64)          40 abits    i32 (activation bits this linear runs with)
  16 N   i32 (rows in this file)    44 crc32    u32 of the image bytes
  20 K   i32                        48 image bytes u64 (= fq_packed_w_bytes(N, K))
  24 N_full i32                     56 k_offset i32 (first weight column of a row-parallel shard)
  28 row_offset i32 (first row of     60 split i32 (0 column-parallel: rows sharded; 1 row-parallel:
     this shard in the rank-major        columns sharded on 128-group boundaries)
     gathered output = rank * N)

Tensor parallelism is FT's decoder layout (`LlamaDecoderLayerWeight.cc:381-410`, flexq_amd.dist):
qkv and gate_up are column-parallel, their parts sharded separately and stacked per rank
(qkv = [q_p; k_p; v_p], gate_up = [gate_p; up_p], FT's per-rank `3 * hidden / tp` layout), so a
rank's attention heads and its gate and up halves stay in its own output; attention.dense and
down_proj are row-parallel (input columns [k_lo, k_hi), the rank's heads / its gate rows), summed
by one all-reduce.  gate/up rows and down columns use the same 128-group split
(dist.group_shard_range).  down_proj runs W6A8 (`--flex_linear_quant`,
int_llama_layer.py:35-37), the others W6A6.

Conversion runs the HIP packer (a GPU is required); reading and writing files does not.
"""
import argparse
import json
import os
import struct
import zlib

import numpy as np
import torch

from . import _lib
from .dist import group_shard_range, shard_range

MAGIC = b"FQW6IMG\0"
VERSION = 1
HEADER = 64
_FMT = "<8sIIiiiiiiiIQii"  # 64 bytes
assert struct.calcsize(_FMT) == HEADER


def packed_bytes(N, K):
    return int(_lib.load().fq_packed_w_bytes(N, K))


def save_image(path, image, N, K, abits, N_full=None, row_offset=0, tp_rank=0, tp_size=1, k_offset=0, split=0):
    """Write one weight image (uint8 tensor of fq_packed_w_bytes(N, K) bytes) with its header."""
    img = image.detach().to("cpu").contiguous().numpy().view(np.uint8).reshape(-1)
    if img.size != packed_bytes(N, K):
        raise ValueError(f"image has {img.size} bytes, expected {packed_bytes(N, K)} for N={N} K={K}")
    if abits not in (6, 8):
        raise ValueError("abits must be 6 or 8")
    hdr = struct.pack(_FMT, MAGIC, VERSION, HEADER, N, K, N if N_full is None else N_full, row_offset,
                      tp_rank, tp_size, abits, zlib.crc32(img) & 0xFFFFFFFF, img.size, k_offset, split)
    tmp = path + ".tmp"
    with open(tmp, "wb") as f:
        f.write(hdr)
        f.write(img.tobytes())
    os.replace(tmp, path)


def read_header(path):
    with open(path, "rb") as f:
        raw = f.read(HEADER)
    if len(raw) != HEADER:
        raise ValueError(f"{path}: truncated header")
    magic, ver, hb, N, K, N_full, off, rank, size, abits, crc, nbytes, k_off, split = struct.unpack(_FMT, raw)
    if magic != MAGIC or ver != VERSION or hb != HEADER:
        raise ValueError(f"{path}: not an fqw6 v{VERSION} file")
    return dict(N=N, K=K, N_full=N_full, row_offset=off, tp_rank=rank, tp_size=size, abits=abits, crc32=crc,
                image_bytes=nbytes, k_offset=k_off, split=split)


def load_image(path, device=None):
    """-> (uint8 image tensor, header dict); checks the size and the CRC of the payload."""
    meta = read_header(path)
    if meta["image_bytes"] != packed_bytes(meta["N"], meta["K"]):
        raise ValueError(f"{path}: image size does not match N={meta['N']} K={meta['K']}")
    img = np.fromfile(path, dtype=np.uint8, offset=HEADER)
    if img.size != meta["image_bytes"]:
        raise ValueError(f"{path}: truncated image ({img.size} of {meta['image_bytes']} bytes)")
    if zlib.crc32(img) & 0xFFFFFFFF != meta["crc32"]:
        raise ValueError(f"{path}: CRC mismatch")
    t = torch.from_numpy(img)
    return (t.to(device) if device is not None else t), meta


def shard_parts(parts, tp_size, tp_rank, by_group=False, return_offset=False):
    """Rows of this rank from each part of a fused linear, stacked: [part0_p; part1_p; ...].
    by_group: rows split on 128-group boundaries (gate/up, matching down_proj's column split).
    With return_offset also the rank's row offset: the rows all lower ranks hold (the sum of the
    parts' shard starts), i.e. where this file's rows begin when the ranks' files are stacked in
    rank order -- exact for uneven group splits (11008 = 86 groups at TP 4: 22/22/21/21)."""
    out, off = [], 0
    for w in parts:
        rng = group_shard_range if by_group else shard_range
        lo, hi = rng(w.shape[0], tp_size, tp_rank)
        out.append(w[lo:hi])
        off += lo
    stacked = torch.cat(out, 0).contiguous()
    return (stacked, off) if return_offset else stacked


def shard_columns(w, tp_size, tp_rank):
    """Columns [k_lo, k_hi) of this rank (row-parallel), split on 128-group boundaries."""
    lo, hi = group_shard_range(w.shape[1], tp_size, tp_rank)
    return w[:, lo:hi].contiguous(), lo


def pack_fp16(w, device):
    """fp16 [N, K] -> weight image on `device` (fq_quantize_pack_w6; needs the GPU)."""
    from . import ops
    wpk, _ = ops.quantize_pack_w6(w.to(device=device, dtype=torch.float16).contiguous())
    return wpk


COLUMN, ROW = 0, 1
LLAMA_LINEARS = [  # (file name, HF parts, activation bits, split)
    ("attention.query_key_value", ("self_attn.q_proj", "self_attn.k_proj", "self_attn.v_proj"), 6, COLUMN),
    ("attention.dense", ("self_attn.o_proj",), 6, ROW),
    ("mlp.gate_up_proj", ("mlp.gate_proj", "mlp.up_proj"), 6, COLUMN),
    ("mlp.down_proj", ("mlp.down_proj",), 8, ROW),
]


def convert_llama_safetensors(src, out_dir, tp_size=1, device="cuda:0", flex_down=True, layers=None):
    """HF LLaMA safetensors (a file or a directory of *.safetensors) -> `.fqw6` files per linear
    and rank + manifest.json.  Returns the manifest dict."""
    from safetensors import safe_open  # no pickle: tensors only
    files = [src] if os.path.isfile(src) else sorted(
        os.path.join(src, f) for f in os.listdir(src) if f.endswith(".safetensors"))
    where = {}
    for fn in files:
        with safe_open(fn, framework="pt") as f:
            for k in f.keys():
                where[k] = fn

    def get(name):
        with safe_open(where[name], framework="pt") as f:
            return f.get_tensor(name)

    n_layers = 1 + max(int(k.split(".")[2]) for k in where if k.startswith("model.layers."))
    if layers is not None:
        n_layers = min(n_layers, layers)
    os.makedirs(out_dir, exist_ok=True)
    manifest = dict(format="fqw6", version=VERSION, tp_size=tp_size, layers=n_layers, linears=[])
    for li in range(n_layers):
        for (fname, parts, ab, split) in LLAMA_LINEARS:
            ws = [get(f"model.layers.{li}.{p}.weight").to(torch.float16) for p in parts]
            K = ws[0].shape[1]
            N_full = sum(w.shape[0] for w in ws)
            abits = ab if flex_down else 6
            for r in range(tp_size):
                k_off = row_off = 0
                if split == ROW:
                    w_r, k_off = shard_columns(ws[0], tp_size, r)
                else:
                    w_r, row_off = shard_parts(ws, tp_size, r, by_group=fname == "mlp.gate_up_proj",
                                               return_offset=True)
                img = pack_fp16(w_r, device)
                path = os.path.join(out_dir, f"model.layers.{li}.{fname}.weight.{r}.fqw6")
                save_image(path, img, w_r.shape[0], w_r.shape[1], abits, N_full=N_full, row_offset=row_off,
                           tp_rank=r, tp_size=tp_size, k_offset=k_off, split=split)
                manifest["linears"].append(dict(layer=li, name=fname, rank=r, N=int(w_r.shape[0]),
                                                K=int(w_r.shape[1]), K_full=int(K), N_full=int(N_full),
                                                abits=abits, parts=list(parts), k_offset=int(k_off),
                                                split="row" if split == ROW else "column",
                                                file=os.path.basename(path)))
    with open(os.path.join(out_dir, "manifest.json"), "w") as f:
        json.dump(manifest, f, indent=1)
    return manifest


def main(argv=None):
    ap = argparse.ArgumentParser(description="HF LLaMA safetensors -> flexq_amd packed W6 weight files")
    ap.add_argument("src", help="a .safetensors file or a directory of them")
    ap.add_argument("out", help="output directory")
    ap.add_argument("--tp", type=int, default=1, help="tensor-parallel ranks (column-parallel shards)")
    ap.add_argument("--device", default="cuda:0")
    ap.add_argument("--no-flex-down", action="store_true", help="down_proj W6A6 instead of W6A8")
    ap.add_argument("--layers", type=int, default=None)
    a = ap.parse_args(argv)
    m = convert_llama_safetensors(a.src, a.out, a.tp, a.device, not a.no_flex_down, a.layers)
    print(f"wrote {len(m['linears'])} files for {m['layers']} layers, tp={a.tp} -> {a.out}")


if __name__ == "__main__":
    main()
