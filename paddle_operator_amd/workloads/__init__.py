"""Workloads a PaddleJob launches through ``pdo-launch`` (BASELINE configs).

* ``gpt2``      — GPT-2(-medium) LM training, collective DP (config 4)
* ``resnet50``  — ResNet-50 image classification, collective DP (configs 2, 3, 5)
* ``wide_deep`` — Wide & Deep CTR, parameter-server mode on CPU (config 1)
* ``deepfm``    — DeepFM CTR (FM + deep over the same sharded tables), PS mode
* ``noop``      — bootstrap + readiness only (launch-latency measurement)

Every workload uses synthetic data of the benchmark's shape and random-init
weights (no network / datasets in this environment).
"""
WORKLOADS = ("gpt2", "resnet50", "wide_deep", "deepfm", "noop")
