"""The perplexity harness with every quantized projection on the HIP W6Ax engine (tiny random
LLaMA, fp16): the engine path runs end to end through FlexQ's evaluate loop and lands within a
percent of the fake-quant accuracy path on the same model."""
import math

import pytest
import torch

from flexq_amd import eval_ppl

pytestmark = pytest.mark.gpu


def test_engine_perplexity_close_to_fake_quant(dev):
    from test_eval_ppl import tiny_llama
    from flexq_amd.flexq_quantize import QuantLinear
    enc = torch.randint(0, 512, (1, 4 * 128), generator=torch.Generator().manual_seed(3))
    ppl = {}
    for engine in (False, True):
        model = tiny_llama(dtype=torch.float16).to(dev)
        if not engine:
            ppl["fp16"] = eval_ppl.perplexity(model, enc, 128)
        eval_ppl.quantize(model, 6, 6, flex_linear_quant=True, engine=engine)
        if engine:
            qls = [m for m in model.modules() if isinstance(m, QuantLinear)]
            assert len(qls) == 14 and all(m.engine for m in qls)
        ppl["engine" if engine else "fake"] = eval_ppl.perplexity(model, enc, 128)
    assert all(math.isfinite(v) for v in ppl.values()), ppl
    assert abs(ppl["engine"] / ppl["fake"] - 1) < 0.01, ppl
    assert abs(ppl["fake"] / ppl["fp16"] - 1) < 0.05, ppl
