"""MI355X-native conv-VAE training hot path (drop-in for parsakzr/medvae-disentangled-multimodal's
src.models / src.losses / VAELightningModule on the training step)."""
from .disentangled import DisentangledConditionalVAE
from .encoder_decoder import AttnBlock, Decoder, Downsample, Encoder, ResnetBlock, Upsample
from .lightning_module import VAELightningModule
from .losses import DisentangledVAELoss, LPIPSLoss, LPIPSWithDiscriminator, VAELoss
from .lpips import LPIPS
from .optim import Adam, AdamW, FlatParameters, FusedAdam
from .schedulers import get_scheduler
from .vae import BaseVAE, BetaVAE, ConditionalVAE

__all__ = ["BaseVAE", "BetaVAE", "ConditionalVAE", "DisentangledConditionalVAE", "DisentangledVAELoss",
           "VAELoss", "LPIPSLoss", "LPIPSWithDiscriminator", "LPIPS", "Encoder", "Decoder", "ResnetBlock", "AttnBlock", "Downsample", "Upsample",
           "VAELightningModule", "FlatParameters", "FusedAdam", "Adam", "AdamW", "get_scheduler"]
