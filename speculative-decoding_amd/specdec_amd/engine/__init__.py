"""Engine package: the batched speculative decode (engine/infer_engine.py) on the HIP path."""
