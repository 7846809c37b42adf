from .attention import Attention, MemEffAttention
from .block import Block, NestedTensorBlock
from .layer_scale import LayerScale
from .mlp import Mlp
from .patch_embed import PatchEmbed
from .rope import PositionGetter, RotaryPositionEmbedding2D
