"""R(2+1)D: network oracle, HIP engine, sampler, decoders and pipeline stages."""
