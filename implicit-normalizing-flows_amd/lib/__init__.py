"""MI355X-native implicit-flow density evaluation, laid out like the reference's ``lib`` package so
train_img.py / train_tabular.py / train_toy.py run on it unchanged (``run_reference.py``).

The modules outside the density path (datasets, optimizers, lr_scheduler, tabular, toy_data, resflow,
visualize_flow) are not re-implemented: they resolve to the reference checkout (``lib._fallthrough``)."""
from . import _fallthrough

_fallthrough.extend_path(__path__)
