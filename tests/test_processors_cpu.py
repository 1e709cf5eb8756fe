"""The processor protocol's extension point (utils/logits_processor.py:7-23).

A subclass of one of the five processors that overrides ``_process`` has it run as written (torch
ops on the rows) and the kernels apply the base class's softmax + sampling rule to its output
(specdec_amd.ops.processed_rows); the GPU loop goldens with such subclasses are in
tests/test_gpu_parity.py (``custom:*`` cases, from the reference itself).  A subclass that redefines
the softmax or the sampling (``__call__`` or ``sample``) is refused with TypeError before anything
runs — never silently executed as its base class.  A subclass that only fixes constructor
parameters is the base processor."""
import pytest
import torch

from custom_procs import make_custom
from specdec_amd import ops
from specdec_amd.ngram_assisted import ngram_assisted_speculative_generate
from specdec_amd.ngram_assisted.ngram_storage import NGramStorage
from specdec_amd.sampling import speculative_generate
from specdec_amd.utils import logits_processor as lp
from specdec_amd.utils.logits_processor import MultinomialProcessor, NucleusProcessor, TopKProcessor
from oracle import specdec_ref as ref


class SharpenedMultinomial(MultinomialProcessor):
    def _process(self, logits):
        return logits * 2.0


class CustomSample(NucleusProcessor):
    def sample(self, probs):
        return probs.argmax(-1, keepdim=True)


class CustomCall(TopKProcessor):
    def __call__(self, logits):
        return logits.softmax(-1)


class Grandchild(SharpenedMultinomial):   # inherits the override from an intermediate class
    pass


class FixedTopK(TopKProcessor):           # parameters only: the base processor
    def __init__(self):
        super().__init__(0.7, 20)


REFUSED = [CustomSample(1.0, 0.9), CustomCall(1.0, 5)]


@pytest.mark.parametrize("proc", REFUSED, ids=lambda p: type(p).__name__)
def test_proc_spec_refuses_sampling_overrides(proc):
    with pytest.raises(TypeError, match="overrides"):
        ops.proc_spec(proc)


@pytest.mark.parametrize("proc", REFUSED, ids=lambda p: type(p).__name__)
def test_drop_in_loops_refuse_sampling_overrides(proc):
    """Both batch-1 loops raise TypeError from the processor check, before touching a model."""
    with pytest.raises(TypeError, match="overrides"):
        speculative_generate([1, 2, 3], None, None, logits_processor=proc, gamma=4)
    with pytest.raises(TypeError, match="overrides"):
        ngram_assisted_speculative_generate([1, 2, 3], NGramStorage(3, 100), None, logits_processor=proc, gamma=4)


@pytest.mark.parametrize("proc", [SharpenedMultinomial(0.8), Grandchild(1.0)], ids=lambda p: type(p).__name__)
def test_process_override_keeps_the_sampling_rule(proc):
    """A _process override: the kernels sample the processed rows with the base's rule, softmax(y / T)."""
    assert ops.proc_spec(proc) == ops.ProcSpec("multinomial", proc.temperature)
    x = torch.randn(2, 16)
    y = ops.processed_rows(proc, x)
    assert torch.equal(y, x * 2.0)
    assert torch.equal(ops.processed_rows(MultinomialProcessor(1.0), x), x)   # the five: rows untouched


@pytest.mark.parametrize("name", ["penalty", "banned_topk", "sharpen_greedy", "nucleus_bias"])
def test_custom_processors_equal_the_oracle(name):
    """The drop-in base classes' torch _process is the reference rule (super() calls in user code):
    processed rows of the test's custom processors equal the oracle's, which runs the same user code
    on the oracle's restatement of the five (tests/custom_procs.py)."""
    x = (torch.randn(3, 4096, generator=torch.Generator().manual_seed(5)) * 3).to(torch.bfloat16)
    ours = make_custom(lp, name, 0.9, 20, 0.9)
    want = make_custom(ref, name, 0.9, 20, 0.9)
    x0 = x.clone()
    y = ops.processed_rows(ours, x)
    assert torch.equal(y, ref.processed_logits(x, want))
    assert torch.equal(x, x0)   # the caller's rows are not modified (banned_topk's base masks in place)
    spec = ops.proc_spec(ours)
    assert spec.kind == ("greedy" if name.endswith("greedy") else "multinomial") and spec.temperature == 0.9


def test_parameter_only_subclass_is_the_base_processor():
    assert ops.proc_spec(FixedTopK()) == ops.ProcSpec("topk", 0.7, 20, 1.0)
    assert ops.proc_spec(MultinomialProcessor(0.5)) == ops.ProcSpec("multinomial", 0.5, 0, 1.0)
    assert ops.processed_rows(FixedTopK(), torch.ones(1, 4)) is not None


def test_unknown_processor_is_refused():
    class Other:
        temperature = 1.0
    with pytest.raises(TypeError, match="unsupported logits processor"):
        ops.proc_spec(Other())
