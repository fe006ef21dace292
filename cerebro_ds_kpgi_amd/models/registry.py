"""MST -> model factory (reference ``create_model_from_mst``,
``cerebro_gpdb/in_rdbms_helper.py:286-426``; ``TorchTrainer.model_fac``,
``cerebro_gpdb/run_pytorchddp.py:295-309``).

Configurations that share an architecture *and* a batch size can be packed
into one horizontally-fused model on a GPU (``pack_key``).

The reference's ``"inceptionresnetv2"`` name silently builds VGG19
(``in_rdbms_helper.py:314-321``); it is kept as an alias of ``vgg19`` so
grids naming it train what the reference actually trained.
``nasnetmobile`` = ``keras.applications.NASNetMobile`` (``models/nasnet.py``);
``squeezenet`` / ``densenet_tf1`` = the raw-TF1 zoo (``models/tf1zoo.py``).
"""

from .mlp import PackedConfA, PackedSanity
from .nasnet import PackedNASNetMobile
from .resnet import PackedResNet
from .small import PackedMobileNetV2, PackedTinyCNN
from .tf1zoo import PackedDenseNetTF1, PackedSqueezeNet
from .vgg import PackedVGG16, PackedVGG16Flat, PackedVGG16Torchvision, PackedVGG19
from .zoo import PackedDenseNet, PackedMobileNetV1, PackedResNeXt, PackedResNet50NoBN

MODEL_FACTORIES = {
    "resnet18": lambda: PackedResNet(18),
    "resnet34": lambda: PackedResNet(34),
    "resnet50": lambda: PackedResNet(50),
    "resnet101": lambda: PackedResNet(101),
    "resnet152": lambda: PackedResNet(152),
    "resnet50_nobn": lambda: PackedResNet50NoBN(),
    "resnext101": lambda: PackedResNeXt(101),
    "vgg16": lambda: PackedVGG16(),
    "vgg19": lambda: PackedVGG19(),
    "vgg16_flat": lambda: PackedVGG16Flat(),
    "vgg16_torchvision": lambda: PackedVGG16Torchvision(),
    "inceptionresnetv2": lambda: PackedVGG19(),
    "densenet121": lambda: PackedDenseNet(121),
    "densenet201": lambda: PackedDenseNet(201),
    "mobilenetv1": lambda: PackedMobileNetV1(),
    "mobilenetv2": lambda: PackedMobileNetV2(),
    "nasnetmobile": lambda: PackedNASNetMobile(),
    "squeezenet": lambda: PackedSqueezeNet(),
    "densenet_tf1": lambda: PackedDenseNetTF1(),
    "confA": lambda: PackedConfA(),
    "sanity": lambda: PackedSanity(),
    "tinycnn": lambda: PackedTinyCNN(),
}


_CUSTOM_DATASETS = {}


def register_model(name, factory, dataset="imagenet"):
    """Add an architecture (a ``PackedNet`` factory) under ``name``; used by
    ``api.schedule`` for user ``model_fn`` callables."""
    MODEL_FACTORIES[name] = factory
    _CUSTOM_DATASETS[name] = dataset
    return name


# PyTorch-DDP baseline (reference run_pytorchddp.py:295-307): its "vgg16" is
# torchvision's; its resnet50 (no conv biases) and confA are ours exactly
TORCH_MODEL_NAMES = {"vgg16": "vgg16_torchvision"}


def create_model_from_mst(mst):
    name = mst["model"]
    if name not in MODEL_FACTORIES:
        raise ValueError("model {} is not available (have: {})".format(
            name, sorted(MODEL_FACTORIES)))
    return MODEL_FACTORIES[name]()


def pack_key(mst):
    """Configs sharing (architecture, batch size, optimizer) pack into one model."""
    return (mst["model"], int(mst["batch_size"]), mst.get("optimizer", "adam"))


def dataset_of(model_name):
    if model_name in _CUSTOM_DATASETS:
        return _CUSTOM_DATASETS[model_name]
    if model_name == "confA":
        return "criteo"
    if model_name == "sanity":
        return "sanity"
    if model_name == "tinycnn":
        return "tiny"
    return "imagenet"
