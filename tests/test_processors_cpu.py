"""The processor protocol's extension point (utils/logits_processor.py:7-23): the kernels fuse the
five processors' arithmetic, so a subclass that redefines behaviour (``__call__``, ``_process`` or
``sample``) is refused with TypeError before anything runs — never silently executed as its base
class.  A subclass that only fixes constructor parameters is the base processor and is accepted."""
import pytest

from specdec_amd import ops
from specdec_amd.ngram_assisted import ngram_assisted_speculative_generate
from specdec_amd.ngram_assisted.ngram_storage import NGramStorage
from specdec_amd.sampling import speculative_generate
from specdec_amd.utils.logits_processor import MultinomialProcessor, NucleusProcessor, TopKProcessor


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


OVERRIDES = [SharpenedMultinomial(1.0), CustomSample(1.0, 0.9), CustomCall(1.0, 5), Grandchild(1.0)]


@pytest.mark.parametrize("proc", OVERRIDES, ids=lambda p: type(p).__name__)
def test_proc_spec_refuses_behaviour_overrides(proc):
    with pytest.raises(TypeError, match="overrides"):
        ops.proc_spec(proc)


@pytest.mark.parametrize("proc", OVERRIDES, ids=lambda p: type(p).__name__)
def test_drop_in_loops_refuse_behaviour_overrides(proc):
    """Both batch-1 loops raise TypeError from the processor check, before touching a model."""
    with pytest.raises(TypeError, match="overrides"):
        speculative_generate([1, 2, 3], None, None, logits_processor=proc, gamma=4)
    with pytest.raises(TypeError, match="overrides"):
        ngram_assisted_speculative_generate([1, 2, 3], NGramStorage(3, 100), None, logits_processor=proc, gamma=4)


def test_parameter_only_subclass_is_the_base_processor():
    assert ops.proc_spec(FixedTopK()) == ops.ProcSpec("topk", 0.7, 20, 1.0)
    assert ops.proc_spec(MultinomialProcessor(0.5)) == ops.ProcSpec("multinomial", 0.5, 0, 1.0)


def test_unknown_processor_is_refused():
    class Other:
        temperature = 1.0
    with pytest.raises(TypeError, match="unsupported logits processor"):
        ops.proc_spec(Other())
