# syntax=docker/dockerfile:1
# Two images from one build (ROCm 7.2 + PyTorch-ROCm base, gfx950 only):
#   pdo/manager   — pdo-manager, pdo-kv, pdo-agent (C++17, no GPU runtime needed)
#   pdo/launcher  — pdo-launch + paddle_operator_amd (HIP kernels for gfx950, RCCL via torch)
ARG BASE=rocm/pytorch:rocm7.2_ubuntu22.04_py3.10_pytorch_2.10

FROM ${BASE} AS build
WORKDIR /src
COPY csrc/ csrc/
COPY tools/ tools/
COPY paddle_operator_amd/ paddle_operator_amd/
COPY __graft_entry__.py setup.cfg* ./
ENV PYTORCH_ROCM_ARCH=gfx950
RUN python3 tools/build.py && ls bin/ paddle_operator_amd/*.so

FROM ubuntu:22.04 AS manager
RUN apt-get update && apt-get install -y --no-install-recommends libstdc++6 ca-certificates && rm -rf /var/lib/apt/lists/*
COPY --from=build /src/bin/pdo-manager /src/bin/pdo-kv /src/bin/pdo-agent /usr/local/bin/
USER 65532:65532
ENTRYPOINT ["/usr/local/bin/pdo-manager"]

FROM ${BASE} AS launcher
WORKDIR /opt/pdo
COPY --from=build /src/paddle_operator_amd/ /opt/pdo/paddle_operator_amd/
COPY --from=build /src/bin/pdo-launch /usr/local/bin/pdo-launch
ENV PYTHONPATH=/opt/pdo HSA_ENABLE_IPC_MODE_LEGACY=0 PDO_PYTHON=python3
ENTRYPOINT ["/usr/local/bin/pdo-launch"]
