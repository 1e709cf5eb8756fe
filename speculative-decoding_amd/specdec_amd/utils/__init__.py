from .logits_processor import (GreedyProcessor, LogitsProcessor, MultinomialProcessor,  # noqa: F401
                               NucleusProcessor, TopKNucleusProcessor, TopKProcessor)
from .caching import prune_cache, prune_dynamic_cache, prune_tuple_cache  # noqa: F401
