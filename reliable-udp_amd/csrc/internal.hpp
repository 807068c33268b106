// Launcher interface between the C ABI (capi.hip) and the kernels.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace rudp {

struct EncodeTileArgs {
  const unsigned char* payload;
  const uint16_t* seq;
  const uint16_t* ack;
  const uint8_t* flags;
  unsigned char* frames;
  uint16_t* csum;       // may be null
  uint64_t n;
  uint32_t L;           // payload bytes per packet
  uint32_t T;           // packets per tile (multiple of 16, power of 2)
  uint32_t glog;        // log2(256 / T): lanes per packet
  uint32_t hdr_bytes;   // LDS bytes reserved for the tile's header words
  uint64_t invF;        // ceil(2^32 / (L + H)) for exact x / F, x < T*F
};

struct DecodeArgs {
  const unsigned char* frames;
  const uint16_t* csum_in;  // rudp5 sideband, may be null
  uint16_t* seq;
  uint16_t* ack;
  uint8_t* flags;
  uint8_t* ok;
  uint16_t* csum_out;       // may be null
  unsigned char* payload_out;  // may be null
  uint64_t n;
  uint32_t F;               // frame bytes
  uint32_t glog;            // log2(lanes per packet)
};

struct SynthArgs {
  uint64_t key_ack, key_flags, key_payload;
  uint32_t isn;
  uint64_t first;
  uint64_t n;
  uint32_t L;
  uint32_t ascii;
  uint16_t* seq;
  uint16_t* ack;
  uint8_t* flags;
  unsigned char* payload;
};

constexpr uint32_t kTileMaxPayload = 4096;

// Tile geometry for a fast-path payload length (L % 16 == 0, 16 <= L <= 4096).
void encode_tile_geometry(uint32_t L, uint32_t* T, uint32_t* glog);
uint32_t decode_group_log2(uint32_t L);

int launch_encode(const EncodeTileArgs& args, int layout, bool tile_path, hipStream_t stream);
int launch_decode(const DecodeArgs& args, int layout, bool vec_path, hipStream_t stream);
int launch_synth(const SynthArgs& args, hipStream_t stream);

}  // namespace rudp
