"""MI355X-native (gfx950) drop-in for the adversarial-attack hot path of
tongxyh/ImageCompression_Adversarial: CompressAI-compatible Balle2018 codecs whose
transforms, GDN, entropy models, MS-SSIM and attack-step updates run as
hand-written HIP kernels behind a C ABI (libica_hip.so)."""
__version__ = "0.1.0"
