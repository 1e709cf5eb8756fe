"""Drop-in for the reference's ``ngram_assisted`` package (rule A11): the n-gram drafters and
the n-gram-assisted speculative loop, with the verify step on the HIP path (sd_ngram_verify)."""
from .ngram_storage import INgramStorage, NGramStorage, OneLevelNGramStorage
from .ngram_assisted import ngram_assisted_speculative_generate
from .device_storage import DeviceNGramStorage, DeviceOneLevelNGramStorage

__all__ = ["INgramStorage", "OneLevelNGramStorage", "NGramStorage", "ngram_assisted_speculative_generate",
           "DeviceOneLevelNGramStorage", "DeviceNGramStorage"]
