"""Experiment catalogs: constants and hyper-parameter grids.

The grids are the reference's experiment definitions, value for value, so
that a grid search run here trains exactly the same configurations:

* ImageNet constants and grids — reference ``cerebro_gpdb/imagenetcat.py:16-105``
* Criteo constants and grids   — reference ``cerebro_gpdb/criteocat.py:15-30``
* images per partition         — reference ``cerebro_gpdb/run_pytorchddp_da.py:32``
* packed-buffer constants      — reference ``cerebro_gpdb/load_imagenet.py:27-32``
"""

SEED = 2018

# ---- ImageNet-112 -------------------------------------------------------
INPUT_SHAPE = (112, 112, 3)
NUM_CLASSES = 1000
TOP_5 = "top_k_categorical_accuracy"
TOP_1 = "categorical_accuracy"
IMAGENET_COUNT_PER_PAR = 160160          # train images per partition (8 partitions)
IMAGENET_TRAIN_TOTAL = 8 * IMAGENET_COUNT_PER_PAR   # 1 281 280
IMAGENET_VALID_TOTAL = 50000
TRAIN_BUFFER_SIZE = 3210                  # images per packed DB buffer
ONE_IMAGE_BYTES = 112 * 112 * 3 * 4       # float32 image in the packed table
# preprocessing normalisation (reference preprocessing/imagenet/generate_h5_file.py:76-81)
IMAGENET_MEAN = (0.485, 0.456, 0.406)
IMAGENET_STD = (0.229, 0.224, 0.225)

# ---- Criteo ---------------------------------------------------------------
INPUT_SHAPE_CRITEO = (7306,)
NUM_CLASSES_CRITEO = 2
CRITEO_TOTAL = 12993256
CRITEO_NUM_CONTINUOUS = 13
CRITEO_NUM_CATEGORICAL = 26
CRITEO_BUCKETS = 50
CRITEO_HASH_BINS = 256
CRITEO_ACTIVE_PER_ROW = CRITEO_NUM_CONTINUOUS + CRITEO_NUM_CATEGORICAL  # 39 ones per row

# ---- grids (imagenetcat.py) ---------------------------------------------
param_grid = {
    "learning_rate": [1e-4, 1e-6],
    "lambda_value": [1e-4, 1e-6],
    "batch_size": [32, 256],
    "model": ["vgg16", "resnet50"],
}

param_grid_hetro = {
    "learning_rate": [1e-4, 1e-4],
    "lambda_value": [1e-4, 1e-4],
    "batch_size": [4, 128],
    "model": ["nasnetmobile", "mobilenetv2"],
    "p": 0.8,
    "hetro": True,
    "fast": 38,
    "slow": 10,
    "total": 48,
}

param_grid_scalability = {
    "learning_rate": [1e-3, 1e-4, 1e-5, 1e-6],
    "lambda_value": [1e-4, 1e-6],
    "batch_size": [32],
    "model": ["resnet50"],
}

param_grid_model_size = {
    "s": {"learning_rate": [1e-4, 1e-6], "lambda_value": [1e-3, 1e-4, 1e-5, 1e-6],
          "batch_size": [32], "model": ["mobilenetv2"]},
    "m": {"learning_rate": [1e-4, 1e-6], "lambda_value": [1e-3, 1e-4, 1e-5, 1e-6],
          "batch_size": [32], "model": ["resnet50"]},
    "l": {"learning_rate": [1e-4, 1e-6], "lambda_value": [1e-3, 1e-4, 1e-5, 1e-6],
          "batch_size": [32], "model": ["resnet152"]},
    "x": {"learning_rate": [1e-4, 1e-6], "lambda_value": [1e-3, 1e-4, 1e-5, 1e-6],
          "batch_size": [32], "model": ["vgg16"]},
}

param_grid_best_model = {
    "learning_rate": [1e-4],
    "lambda_value": [1e-4],
    "batch_size": [32],
    "model": ["resnet50"],
}

# hyperopt search space: lr ~ logU[lo, hi], batch in [lo, hi], choices otherwise
param_grid_hyperopt = {
    "learning_rate": [0.00001, 0.1],
    "lambda_value": [1e-4, 1e-6],
    "batch_size": [16, 256],
    "model": ["resnet18", "resnet34"],
}

# ---- grids (criteocat.py) -------------------------------------------------
param_grid_criteo = {
    "learning_rate": [1e-3, 1e-4],
    "lambda_value": [1e-4, 1e-5],
    "batch_size": [32, 64, 256, 512],
    "model": ["confA"],
}

param_grid_criteo_breakdown = {
    "learning_rate": [1e-3, 1e-4],
    "lambda_value": [1e-3, 1e-4, 1e-5, 1e-6],
    "batch_size": [256],
    "model": ["confA"],
}

# New (BASELINE config 4): heterogeneous {ResNet-50, VGG-16} x {lr, batch} 8-config MOP.
param_grid_hetero_rv = {
    "learning_rate": [1e-3, 1e-4],
    "lambda_value": [1e-4],
    "batch_size": [32, 64],
    "model": ["resnet50", "vgg16"],
}

# New (BASELINE config 1): tiny CNN on 32x32 synthetic images, CPU plumbing test.
param_grid_tiny = {
    "learning_rate": [1e-3, 1e-2],
    "lambda_value": [1e-4],
    "batch_size": [8],
    "model": ["tinycnn"],
}

# DB-era names kept so that log tables / experiment labels read the same.
MODEL_ARCH_TABLE = "model_arch_library"
MODEL_SELECTION_TABLE = "mst_table"
MODEL_SELECTION_SUMMARY_TABLE = "mst_table_summary"
