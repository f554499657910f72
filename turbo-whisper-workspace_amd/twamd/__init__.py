"""twamd — MI355X-native Whisper batch-transcription hot path (drop-in for the reference's ASR callable).

Layers:
  csrc/ (libtwhip.so, C-ABI in include/tw_whisper.h)  HIP kernels for gfx950
  _lib        ctypes binding, fails loudly if the library is missing
  engine      WhisperEngine: weights + activations in HBM, encoder / decoder / seek loop
  pipeline    TurboTranscriber: the HF-pipeline-compatible callable
  audio_pipeline  AudioProcessingPipeline mirror (transcribe / process_audio / load_transcription_model)
  dist        chunk data-parallelism over RCCL (one process per GPU)
"""
__version__ = "0.1.0"

from .config import PRESETS, GenerationSettings, SpecialTokens, WhisperDims  # noqa: F401
