"""CPU tests of the perplexity harness (flexq_amd/eval_ppl.py; FlexQ's evaluate, main.py:84-126)
on a tiny random-init LLaMA: the loop equals the model's own loss, the reference's quantization
flow runs through it, and local data loading (text, parquet, save_to_disk, git-lfs stubs)."""
import math
import os

import pytest
import torch

from flexq_amd import eval_ppl


def tiny_llama(seed=0, dtype=torch.float32):
    from transformers import LlamaConfig, LlamaForCausalLM
    torch.manual_seed(seed)
    cfg = LlamaConfig(vocab_size=512, hidden_size=256, intermediate_size=512, num_hidden_layers=2,
                      num_attention_heads=2, num_key_value_heads=2, max_position_embeddings=256)
    return LlamaForCausalLM(cfg).to(dtype).eval()


def test_perplexity_matches_the_models_own_loss():
    model = tiny_llama()
    g = torch.Generator().manual_seed(1)
    enc = torch.randint(0, 512, (1, 4 * 64 + 17), generator=g)  # 4 windows + a ragged tail (dropped)
    ppl = eval_ppl.perplexity(model, enc, 64)
    with torch.no_grad():
        losses = [model(enc[:, i * 64:(i + 1) * 64], labels=enc[:, i * 64:(i + 1) * 64]).loss for i in range(4)]
    assert ppl == pytest.approx(math.exp(torch.stack(losses).mean().item()), rel=1e-5)
    assert eval_ppl.perplexity(model, enc, 64, limit=2) == pytest.approx(math.exp(torch.stack(losses[:2]).mean().item()),
                                                                         rel=1e-5)
    with pytest.raises(ValueError):
        eval_ppl.perplexity(model, enc[:, :10], 64)


def test_quantized_flow_runs_through_the_loop():
    from flexq_amd.flexq_quantize import QuantLinear
    model = tiny_llama()
    enc = torch.randint(0, 512, (1, 3 * 64), generator=torch.Generator().manual_seed(2))
    ppl = eval_ppl.perplexity(model, enc, 64)
    eval_ppl.quantize(model, 6, 6, flex_linear_quant=True)
    n = sum(isinstance(m, QuantLinear) for m in model.modules())
    assert n == 2 * 7  # q, k, v, o, gate, up, down per layer
    downs = [m for name, m in model.named_modules() if name.endswith("down_proj")]
    assert all(m.act_quantizer.n_bits == 8 for m in downs)  # --flex_linear_quant: W6A8 down_proj
    model.float()
    pq = eval_ppl.perplexity(model, enc, 64)
    assert math.isfinite(pq) and abs(pq / ppl - 1) < 0.05


def test_load_text_formats(tmp_path):
    lines = ["= Title =", "", "Some text .", "More text"]
    txt = tmp_path / "wiki.txt"
    txt.write_text("\n\n".join(lines))
    assert eval_ppl.load_text(str(txt)) == "\n\n".join(lines)
    import pyarrow as pa
    import pyarrow.parquet as pq
    pq.write_table(pa.table({"text": lines}), str(tmp_path / "test.parquet"))
    assert eval_ppl.load_text(str(tmp_path / "test.parquet")) == "\n\n".join(lines)
    import datasets
    datasets.DatasetDict({"test": datasets.Dataset.from_dict({"text": lines})}).save_to_disk(str(tmp_path / "ds"))
    assert eval_ppl.load_text(str(tmp_path / "ds")) == "\n\n".join(lines)


def test_lfs_pointer_stubs_are_reported(tmp_path):
    d = tmp_path / "stub" / "test"
    d.mkdir(parents=True)
    (d / "data-00000-of-00001.arrow").write_text(
        "version https://git-lfs.github.com/spec/v1\noid sha256:00\nsize 1\n")
    with pytest.raises(FileNotFoundError, match="git-lfs"):
        eval_ppl.load_text(str(tmp_path / "stub"))
    ref = "/root/reference/datasets/wikitext-2-raw-v1"  # the reference's copy (this container only)
    if os.path.isdir(ref):
        with pytest.raises(FileNotFoundError, match="git-lfs"):
            eval_ppl.load_text(ref)
