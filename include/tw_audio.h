/*
 * tw_audio.h — C-ABI of the native audio ingest in front of the transcription hot path.
 *
 * The reference reads every input through ffmpeg: transformers' ffmpeg_read
 * ($TF/pipelines/audio_utils.py:9-45, called from AutomaticSpeechRecognitionPipeline.preprocess,
 * $TF/pipelines/automatic_speech_recognition.py:345-356) pipes the file bytes through
 * `ffmpeg -i pipe:0 -ac 1 -ar 16000 -f f32le`, i.e. container decode -> downmix to mono -> libswresample's
 * default resampler -> float32. This image has no ffmpeg, so these two stages are native here:
 *
 *   tw_flac_probe / tw_flac_decode   FLAC container + frame decode on HOST memory (multi-threaded over frames),
 *                                    bit-exact PCM (checked against the stream's own STREAMINFO MD5)
 *   tw_g711_decode                   G.711 mu-law / A-law expansion (WAV, AU, AIFF-C telephony codecs)
 *   tw_ima_adpcm_wav_decode          IMA ADPCM in WAV blocks
 *   tw_ms_adpcm_wav_decode           Microsoft ADPCM in WAV blocks
 *   tw_ima_qt_decode                 Apple IMA4 (AIFF-C 'ima4')
 *   tw_vorbis_probe / tw_vorbis_decode  Ogg Vorbis I (floor 1, residues 0/1/2, coupling, IMDCT, overlap-add)
 *   tw_mp3_probe / tw_mp3_decode     MPEG-1 / MPEG-2 LSF / MPEG-2.5 Layer III (MP3), gapless-trimmed by the
 *                                    LAME tag as ffmpeg's mp3 demuxer trims it, and Layers I / II
 *   tw_aac_*                         MPEG-4 AAC-LC: ADTS streams, and the raw access units of an MP4 / M4A track
 *   tw_alac_*                        Apple Lossless access units of an MP4 / M4A track
 *                                    (the container is demuxed by the caller, twamd/audio.py)
 *   tw_resample_pcm_i32 / _f32       downmix + polyphase resample on the GPU (DEVICE memory, `stream`), the
 *                                    libswresample default filter restated (Kaiser-windowed sinc, see
 *                                    twamd/audio.py: swr_filter_bank)
 *
 * Conventions as tw_whisper.h: 0 = success, nonzero = failure with tw_last_error() set.
 */
#ifndef TW_AUDIO_H
#define TW_AUDIO_H
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct TwFlacInfo {
  int32_t sample_rate;     /* Hz (STREAMINFO)                                                          */
  int32_t channels;        /* 1..8                                                                     */
  int32_t bits_per_sample; /* 4..32                                                                    */
  int32_t min_blocksize;   /* samples per channel                                                      */
  int32_t max_blocksize;
  int32_t total_from_frames; /* 1: STREAMINFO's total was 0 (unknown) and total_samples comes from the last frame */
  int64_t total_samples;   /* per channel; 0 = unknown and no frame found (tw_flac_decode refuses the stream) */
  int64_t audio_offset;    /* byte offset of the first frame                                           */
  uint8_t md5[16];         /* MD5 of the unencoded PCM (interleaved, little-endian, ceil(bps/8) bytes) */
} TwFlacInfo;

/* Parse the "fLaC" marker and the metadata blocks (STREAMINFO required). HOST memory. A STREAMINFO total of 0
 * (unknown: a stream written to a pipe) is replaced by the last genuine frame's first sample + block size
 * (total_from_frames = 1), as ffmpeg decodes such a stream to its end. */
int tw_flac_probe(const uint8_t* data, int64_t size, TwFlacInfo* info);

/* Decode every frame into out = int32[out_frames][channels] (interleaved, HOST memory, sample values as coded,
 * i.e. in [-2^(bps-1), 2^(bps-1))). out_frames must be >= info.total_samples. Frames are verified with their
 * CRC-8 header and CRC-16 footer; a damaged frame is an error (no concealment). n_threads <= 0 = hardware
 * concurrency. *frames_decoded receives the samples per channel written. */
int tw_flac_decode(const uint8_t* data, int64_t size, int32_t* out, int64_t out_frames, int32_t n_threads,
                   int64_t* frames_decoded);

/* Polyphase resampling y[n] = sum_i taps[ph][i] * x[idx + i - center], idx = floor(n*down/up),
 * ph = (n*down) % up, center = (ntaps-1)/2, x reflected at both ends (x[-k] = x[k], x[n_in-1+k] = x[n_in-1-k]).
 * taps: f32[up][ntaps] DEVICE. y: f32[n_out] DEVICE.
 *   _i32: x[t] = scale * mean_c pcm[t][c]   (pcm int32[n_in][channels], DEVICE)  — decode output as-is
 *   _f32: x[t] = mean_c x_in[t][c]           (f32[n_in][channels], DEVICE)
 * up == down == 1 with ntaps == 1 is a plain downmix/convert. */
int tw_resample_pcm_i32(const int32_t* pcm, int64_t n_in, int32_t channels, float scale, int32_t up, int32_t down,
                        const float* taps, int32_t ntaps, float* y, int64_t n_out, void* stream);
int tw_resample_pcm_f32(const float* x, int64_t n_in, int32_t channels, int32_t up, int32_t down, const float* taps,
                        int32_t ntaps, float* y, int64_t n_out, void* stream);

/* G.711 expansion of n codes to s16 (HOST memory): mu-law (alaw == 0) or A-law, the classic ITU-T G.711 tables
 * (WAV format tags 7 / 6, AU encodings 1 / 27, AIFF-C 'ulaw' / 'alaw'; what ffmpeg_read's pcm_mulaw / pcm_alaw give). */
int tw_g711_decode(const uint8_t* in, int64_t n, int32_t alaw, int16_t* out);

/* IMA ADPCM in Microsoft's WAV block layout (format tag 0x11, 4 bits per sample; ffmpeg's adpcm_ima_wav): blocks of
 * block_align bytes (the last may be shorter), each channel's 4-byte header {s16 first sample, u8 step index, u8 0},
 * then 4-byte words of 8 samples per channel, interleaved, low nibble first. out = int16[out_frames][channels]
 * interleaved (HOST); *frames_decoded receives the frames written (1 + 8 * whole words per channel per block). */
int tw_ima_adpcm_wav_decode(const uint8_t* data, int64_t size, int32_t channels, int32_t block_align, int16_t* out,
                            int64_t out_frames, int64_t* frames_decoded);

/* Microsoft ADPCM in WAV blocks (format tag 2; ffmpeg's adpcm_ms), 1 or 2 channels: per block the channels'
 * predictor indices (u8, the standard seven coefficient pairs), s16 deltas, s16 sample1 and s16 sample2, then two
 * nibbles per byte, high first. A block of L bytes gives (L - 6 channels) * 2 / channels frames (the last may be
 * shorter); a block naming a predictor index > 6 is dropped, as ffmpeg drops a packet it cannot decode. out =
 * int16[out_frames][channels] interleaved (HOST). */
int tw_ms_adpcm_wav_decode(const uint8_t* data, int64_t size, int32_t channels, int32_t block_align, int16_t* out,
                           int64_t out_frames, int64_t* frames_decoded);

/* Apple IMA4 (AIFF-C / QuickTime 'ima4'; ffmpeg's adpcm_ima_qt): packets of 34 bytes per channel, 64 frames each;
 * a channel's IMA state carries over a packet boundary as ffmpeg carries it (same step index, predictor within
 * 0x7f), otherwise the packet header resets it. out = int16[out_frames][channels] interleaved (HOST). */
int tw_ima_qt_decode(const uint8_t* data, int64_t size, int32_t channels, int16_t* out, int64_t out_frames,
                     int64_t* frames_decoded);

typedef struct TwAlacInfo {
  int32_t sample_rate;   /* Hz (ALACSpecificConfig)                                                    */
  int32_t channels;      /* 1 or 2 (other layouts are refused)                                          */
  int32_t bit_depth;     /* 16, 20, 24 or 32                                                            */
  int32_t frame_length;  /* samples per full frame (4096 from Apple's encoder)                          */
  int32_t pb, mb, kb;    /* Rice history multiplier, initial history, parameter limit                   */
} TwAlacInfo;

/* Apple Lossless (ALAC) in an MP4 / M4A track (HOST memory; ffmpeg's alac decoder): `cookie` is the track's
 * ALACSpecificConfig (24 bytes, or the 36-byte 'alac' atom holding it). */
int tw_alac_parse_cookie(const uint8_t* cookie, int64_t size, TwAlacInfo* info);

/* Decode the n_packets access units at data + offsets[k] (sizes[k] bytes each; the caller demuxes the container)
 * into out = f32[out_frames][channels], interleaved, sample / 2^(bit_depth - 1). A packet whose first element
 * header is invalid, or that the decoder refuses, contributes no samples (ffmpeg drops it). Packets decode on
 * n_threads threads (<= 0: hardware concurrency); frames are independent, so the output does not depend on it.
 * *frames_decoded receives the frames written. */
int tw_alac_decode(const uint8_t* cookie, int64_t cookie_size, const uint8_t* data, int64_t size,
                   const int64_t* offsets, const int64_t* sizes, int64_t n_packets, float* out, int64_t out_frames,
                   int32_t n_threads, int64_t* frames_decoded);

typedef struct TwVorbisInfo {
  int32_t sample_rate;   /* Hz (identification header)                                            */
  int32_t channels;      /* 1..16                                                                 */
  int32_t blocksize0;    /* short / long MDCT block sizes                                         */
  int32_t blocksize1;
  int64_t total_samples; /* per channel: the granule position of the stream's last audio page      */
} TwVorbisInfo;

/* Ogg Vorbis I (HOST memory; the first logical stream of the file): check the Ogg pages (CRC-32) and parse the
 * identification, comment and setup headers. Floor type 0 streams are refused with an error. */
int tw_vorbis_probe(const uint8_t* data, int64_t size, TwVorbisInfo* info);

/* Decode every audio packet into out = f32[out_frames][channels] (interleaved, HOST; the codec's own scale,
 * nominally [-1, 1]). out_frames must be >= info.total_samples. The first packet primes the overlap (no output);
 * the end is trimmed to the last page's granule position. Packets decode on n_threads threads (<= 0: hardware
 * concurrency; the output does not depend on it), the overlap-add runs in order. *frames_decoded receives the
 * frames written. */
int tw_vorbis_decode(const uint8_t* data, int64_t size, float* out, int64_t out_frames, int32_t n_threads,
                     int64_t* frames_decoded);

/* The Vorbis inverse MDCT alone (for tests): y[i] = sum_{k < n/2} X[k] cos(2 pi / n (i + 1/2 + n/4)(k + 1/2)),
 * i < n, n a power of two >= 4. HOST memory. */
int tw_vorbis_imdct(const float* X, int32_t n, float* y);

typedef struct TwMp3Info {
  int32_t sample_rate;       /* Hz (first audio frame; the stream may not change rate or channel count)      */
  int32_t channels;          /* 1 or 2                                                                        */
  int32_t version;           /* 1 (MPEG-1), 2 (MPEG-2 LSF) or 25 (MPEG-2.5)                                  */
  int32_t bitrate_kbps;      /* of the first audio frame                                                      */
  int64_t total_samples;     /* per channel, after the gapless trim (all decoded samples without a LAME tag)  */
  int64_t n_frames;          /* audio frames (a Xing / Info / VBRI header frame is not counted)               */
  int64_t skip_samples;      /* decoded samples dropped at the start (LAME delay + 529; 0 without the tag)    */
  int32_t samples_per_frame; /* 1152 (Layer II, MPEG-1 Layer III), 576 (LSF Layer III) or 384 (Layer I)       */
  int32_t enc_delay;         /* LAME / Lavc tag encoder delay and padding (-1: no such tag)                   */
  int32_t enc_padding;
  int32_t flags;             /* 1: Xing / Info frame, 2: LAME gapless fields, 4: VBRI frame                  */
  int32_t layer;             /* 1, 2 or 3 (a stream does not change layer)                                    */
} TwMp3Info;

/* MP3 / MPEG audio (HOST memory): skip ID3v2 tags, find the first frame (Layer I, II or III) the next header
 * confirms, walk the frames of that layer (resynchronising over junk, stopping at ID3v1 / APEv2 / trailing ID3 tags)
 * and, for Layer III, read the Xing / Info + LAME or VBRI header frame. Free-format streams are refused.
 * Reference: the codec half of ffmpeg_read ($TF/pipelines/audio_utils.py:9-45) for the .mp3 uploads
 * vocalis/api/main.py:67-75 stores. */
int tw_mp3_probe(const uint8_t* data, int64_t size, TwMp3Info* info);

/* Decode into out = f32[out_frames][channels] (interleaved, HOST, nominal full scale +-1). out_frames must be >=
 * info.total_samples. Frame ranges decode on n_threads threads (<= 0: hardware concurrency), each primed by the
 * frame before its range: the output does not depend on the thread count. A frame whose reservoir reaches before
 * the first frame, or whose side information is reserved, decodes as silence. *frames_decoded receives the frames
 * written (= info.total_samples). */
int tw_mp3_decode(const uint8_t* data, int64_t size, float* out, int64_t out_frames, int32_t n_threads,
                  int64_t* frames_decoded);

typedef struct TwAacInfo {
  int32_t sample_rate;   /* Hz                                                                          */
  int32_t channels;      /* of the channel configuration (1..7 -> 1, 2, 3, 4, 5, 6, 8)                  */
  int32_t object_type;   /* 2 (LC): every other object type is refused                                  */
  int32_t frame_length;  /* 1024                                                                        */
  int64_t n_frames;      /* ADTS: frames found (0 for tw_aac_parse_asc)                                 */
  int64_t total_samples; /* n_frames * 1024 per channel (no trim)                                       */
} TwAacInfo;

/* The AudioSpecificConfig of an MP4 track (esds DecoderSpecificInfo). Refused: object types other than LC, HE-AAC
 * (SBR / PS, explicit or backward-compatible signalling), 960-sample frames, channel configuration 0. */
int tw_aac_parse_asc(const uint8_t* asc, int32_t asc_size, TwAacInfo* info);

/* Decode n_au raw access units data[au_offset[i] .. + au_size[i]) (HOST) of the stream asc describes into
 * out = f32[out_frames][channels] (interleaved, nominal full scale +-1), 1024 samples per unit, untrimmed (an MP4 edit
 * list is applied by the caller). out_frames >= n_au * 1024. Units decode on n_threads threads (<= 0: hardware
 * concurrency), each range primed by the unit before it: the output does not depend on the thread count. Every unit
 * must parse to its END element (an error names the unit). Replaces ffmpeg_read's AAC decode
 * ($TF/pipelines/audio_utils.py:9-45) for the .m4a uploads vocalis/security/security_monitor.py:353 lists. */
int tw_aac_decode_raw(const uint8_t* asc, int32_t asc_size, const uint8_t* data, int64_t size, const int64_t* au_offset,
                      const int64_t* au_size, int64_t n_au, float* out, int64_t out_frames, int32_t n_threads,
                      int64_t* frames_decoded);

/* ADTS (.aac): skip ID3v2 tags, find the first frame, walk the frames of the same stream (one raw_data_block per
 * frame; CRC words skipped). */
int tw_aac_adts_probe(const uint8_t* data, int64_t size, TwAacInfo* info);
int tw_aac_adts_decode(const uint8_t* data, int64_t size, float* out, int64_t out_frames, int32_t n_threads,
                       int64_t* frames_decoded);

#ifdef __cplusplus
}
#endif
#endif
