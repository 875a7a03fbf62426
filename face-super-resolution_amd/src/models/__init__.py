"""Model API of the reference (src/models/__init__.py:1-36), restricted to the FaceEnhanceNet
hot path: `from src.models import FaceEnhanceNet, FaceEnhanceNetConfig, create_face_enhance_net,
FaceEnhanceNetLite, RCAB, ChannelAttention, ResidualGroup, UpsampleModule`.  The ESRGAN,
transfer and discriminator models are outside this build's scope."""
from .blocks import (RCAB, ChannelAttention, PixelShuffleUpsample, ResidualGroup, UpsampleModule, icnr_init,
                     initialize_weights)
from .custom import FaceEnhanceNet, FaceEnhanceNetConfig, FaceEnhanceNetLite, create_face_enhance_net
from .discriminator import GANLoss, VGGStyleDiscriminator, create_discriminator

__all__ = [
    "VGGStyleDiscriminator", "GANLoss", "create_discriminator",
    "FaceEnhanceNet", "FaceEnhanceNetLite", "FaceEnhanceNetConfig", "create_face_enhance_net",
    "RCAB", "ChannelAttention", "UpsampleModule", "ResidualGroup", "PixelShuffleUpsample",
    "icnr_init", "initialize_weights",
]
