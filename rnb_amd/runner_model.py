"""Stage plugin contract (reference: runner_model.py:1-81).

A pipeline step is a ``RunnerModel``:

* ``__init__(device, **kwargs)`` builds the stage on ``device`` (a
  ``torch.device``; ``cpu`` when the config lists gpu ``-1``);
* ``input_shape()`` returns the nested tuple of expected input shapes, or
  ``None`` if the stage takes no tensors;
* ``output_shape()`` (static) returns the nested tuple of output shapes used
  to size the inter-stage slot rings, or ``None``;
* ``output_dtypes()`` (static, optional, rnb_amd addition) returns one torch
  dtype per output tensor; the default is float32 like the reference;
* ``__call__(tensors, non_tensors, time_card) -> (tensors, non_tensors,
  time_card)``. Returning ``None`` as the time card means "no output yet"
  (batching / aggregation).

``flush()`` (optional, rnb_amd addition) is called once at the natural end
of the input stream and may return one last ``(tensors, non_tensors,
time_card)`` (e.g. a partial batch), or ``None``.

``output_shape_for(**kwargs)`` (rnb_amd addition) may be overridden when the
slot shape depends on step kwargs, which fixes the reference's TODO #69
(model.py:76-80: partial R(2+1)D runners always advertised ``(10, 400)``).
"""


class RunnerModel:
    def __init__(self, device, **kwargs):
        self.device = device

    def input_shape(self):
        raise NotImplementedError

    @staticmethod
    def output_shape():
        raise NotImplementedError

    @staticmethod
    def output_dtypes():
        return None

    @classmethod
    def output_shape_for(cls, **kwargs):
        """Output shapes given the step kwargs (defaults to output_shape())."""
        return cls.output_shape()

    @classmethod
    def output_dtypes_for(cls, **kwargs):
        return cls.output_dtypes()

    def __call__(self, tensors, non_tensors, time_card):
        raise NotImplementedError
