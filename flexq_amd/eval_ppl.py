"""WikiText-2 perplexity loop for the FlexQ accuracy claim (<= +0.1 PPL over fp16,
README.md:14), restating FlexQ's `evaluate` (algorithm/main.py:84-126):

    testenc  = tokenizer("\\n\\n".join(test["text"]))                        (datautils.py:30-35)
    nsamples = numel // seqlen
    for i:   logits = lm_head(model.model(testenc[:, i*seqlen:(i+1)*seqlen])[0])
             nll_i  = CrossEntropy(logits[:, :-1], tokens[:, 1:]) * seqlen
    ppl      = exp(sum(nll) / (n * seqlen))

The model runs in fp16 first, then through this build's `flexqllm` (the reference's flag
mapping, QuantLinear per projection, weight_quant_inplace) and -- with --engine -- with every
eligible QuantLinear on the HIP W6Ax engine (dynamic A6 / A8 quantization + int8-MFMA GEMM).

Everything is read locally and nothing is fetched: --model is a local HF model directory
(weights + tokenizer, `local_files_only`), --data a local WikiText-2 copy (a `datasets`
save_to_disk directory, a .parquet or a .txt file).  The copy at
/root/reference/datasets/wikitext-2-raw-v1 holds git-lfs pointer stubs instead of arrow data;
`load_text` recognises them and says so.

usage: python -m flexq_amd.eval_ppl --model DIR --data PATH [--wbits 6 --abits 6 --flex_linear_quant
       --engine --seqlen 2048 --limit N]
"""
import argparse
import json
import math
import os

import torch
import torch.nn as nn


def _lfs_pointer(path):
    try:
        with open(path, "rb") as f:
            head = f.read(64)
    except OSError:
        return False
    return head.startswith(b"version https://git-lfs.github.com/spec/")


def load_text(path, split="test"):
    """The split's text joined as FlexQ joins it ("\\n\\n", datautils.py:33-34)."""
    if os.path.isdir(path):
        sub = os.path.join(path, split)
        root = sub if os.path.isdir(sub) else path
        arrows = sorted(f for f in os.listdir(root) if f.endswith(".arrow"))
        for f in arrows:
            if _lfs_pointer(os.path.join(root, f)):
                raise FileNotFoundError(f"{os.path.join(root, f)} is a git-lfs pointer, not arrow data: the "
                                        "dataset was checked out without its large files")
        import datasets
        ds = datasets.load_from_disk(path)
        texts = (ds[split] if isinstance(ds, datasets.DatasetDict) else ds)["text"]
    elif path.endswith(".parquet"):
        import pyarrow.parquet as pq
        texts = pq.read_table(path).column("text").to_pylist()
    else:
        if _lfs_pointer(path):
            raise FileNotFoundError(f"{path} is a git-lfs pointer")
        with open(path, encoding="utf-8") as f:
            return f.read()
    return "\n\n".join(texts)


@torch.no_grad()
def perplexity(model, testenc, seqlen, limit=-1, device=None):
    """main.py:98-126 for a LLaMA-style HF causal LM (model.model -> hidden states, lm_head).
    limit > 0 stops after `limit` windows; the mean then runs over the windows evaluated (the
    reference divides by all nsamples even when --limit cuts the loop short)."""
    device = device or next(model.parameters()).device
    nsamples = testenc.numel() // seqlen
    if nsamples == 0:
        raise ValueError(f"{testenc.numel()} tokens do not fill one window of {seqlen}")
    use_cache = getattr(model.config, "use_cache", None)
    model.config.use_cache = False
    model.eval()
    nlls = []
    loss_fct = nn.CrossEntropyLoss()
    for i in range(nsamples):
        batch = testenc[:, i * seqlen:(i + 1) * seqlen].to(device)
        hidden = model.model(batch)[0]
        logits = model.lm_head(hidden)
        shift_logits = logits[:, :-1, :]
        shift_labels = batch[:, 1:]
        loss = loss_fct(shift_logits.reshape(-1, shift_logits.size(-1)).float(), shift_labels.reshape(-1))
        nlls.append(loss.float() * seqlen)
        if limit > 0 and len(nlls) >= limit:
            break
    if use_cache is not None:
        model.config.use_cache = use_cache
    return math.exp(torch.stack(nlls).sum().item() / (len(nlls) * seqlen))


def quantize(model, wbits=6, abits=6, flex_linear_quant=True, engine=False, group=128):
    """The reference flow on `model` in place: main.py's flag mapping (--wbits --abits
    --w_group_size 128 --a_group_size 128 --symmetric [--flex_linear_quant]) and flexqllm."""
    from .flexq_quantize import build_quant_params, flexqllm, make_arg_parser
    args = make_arg_parser().parse_args(["--wbits", str(wbits), "--abits", str(abits), "--w_group_size", str(group),
                                         "--a_group_size", str(group), "--symmetric"]
                                        + (["--flex_linear_quant"] if flex_linear_quant else [])
                                        + (["--engine"] if engine else []))
    build_quant_params(args)
    return flexqllm(model, args)


def main(argv=None):
    ap = argparse.ArgumentParser(description="WikiText-2 perplexity, fp16 vs FlexQ W6Ax (local files only)")
    ap.add_argument("--model", required=True, help="local HF causal-LM directory (weights + tokenizer)")
    ap.add_argument("--data", required=True, help="local WikiText-2 (save_to_disk dir, .parquet or .txt)")
    ap.add_argument("--wbits", type=int, default=6)
    ap.add_argument("--abits", type=int, default=6)
    ap.add_argument("--flex_linear_quant", action="store_true", help="down_proj W6A8")
    ap.add_argument("--engine", action="store_true", help="quantized linears on the HIP engine")
    ap.add_argument("--seqlen", type=int, default=2048)
    ap.add_argument("--limit", type=int, default=-1)
    ap.add_argument("--device", default="cuda:0")
    a = ap.parse_args(argv)
    from transformers import AutoModelForCausalLM, AutoTokenizer
    tok = AutoTokenizer.from_pretrained(a.model, local_files_only=True, use_fast=False)
    model = AutoModelForCausalLM.from_pretrained(a.model, local_files_only=True, torch_dtype=torch.float16)
    model.to(a.device)
    testenc = tok(load_text(a.data), return_tensors="pt").input_ids
    ppl16 = perplexity(model, testenc, a.seqlen, a.limit)
    quantize(model, a.wbits, a.abits, a.flex_linear_quant, a.engine)
    pplq = perplexity(model, testenc, a.seqlen, a.limit)
    print(json.dumps({"dataset": "wikitext2", "seqlen": a.seqlen, "windows": testenc.numel() // a.seqlen,
                      "limit": a.limit, "ppl_fp16": ppl16, f"ppl_w{a.wbits}a{a.abits}": pplq,
                      "delta": pplq - ppl16, "engine": a.engine, "target_delta": 0.1}))


if __name__ == "__main__":
    main()
