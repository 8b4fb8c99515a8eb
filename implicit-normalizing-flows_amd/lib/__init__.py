"""MI355X-native implicit-flow density evaluation, laid out like the reference's ``lib`` package so
train_img.py / train_tabular.py style code can ``import lib.layers as layers`` unchanged."""
