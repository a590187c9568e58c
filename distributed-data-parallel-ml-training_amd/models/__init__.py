"""Model zoo: VGG-11/13/16/19 (reference family) and ResNet-50 (driver's large-gradient config)."""
from .vgg import VGG11, VGG13, VGG16, VGG19, _VGG  # noqa: F401


def build(name):
    name = name.lower()
    table = {"vgg11": VGG11, "vgg13": VGG13, "vgg16": VGG16, "vgg19": VGG19}
    if name in table:
        return table[name]()
    if name in ("resnet50", "resnet-50"):
        from .resnet import resnet50
        return resnet50()
    raise ValueError(f"unknown model {name}")
