# MI355X serving image.  The base carries ROCm 7 + PyTorch-ROCm; the HIP kernels
# are compiled for gfx950 at image build time (no JIT at start-up).
#
#   docker build -t rfq-mi355x .
#   docker run --device=/dev/kfd --device=/dev/dri --group-add video \
#       --ipc=host -e RFQ_MODEL=llama3-8b -e RFQ_DP=8 -p 8000:8000 rfq-mi355x
ARG BASE=rocm/pytorch:latest
FROM ${BASE}

WORKDIR /srv/rfq
ENV PYTHONUNBUFFERED=1 \
    PYTORCH_ROCM_ARCH=gfx950 \
    HSA_ENABLE_IPC_MODE_LEGACY=0

COPY requirements.txt ./
RUN pip install --no-cache-dir -r requirements.txt

COPY csrc/ csrc/
COPY replisense_rfq_amd/ replisense_rfq_amd/
COPY __graft_entry__.py bench.py ./
COPY tools/ tools/
RUN python -c "from replisense_rfq_amd._build import build_all; build_all()" \
 && mkdir -p uploads

EXPOSE 8000
# One API process; RFQ_DP>1 spawns one engine replica per GPU (or per TP group
# of RFQ_TP GPUs) behind the in-process router.
CMD ["python", "-m", "replisense_rfq_amd.api.serve", "--host", "0.0.0.0", "--port", "8000"]
