from .registry import (MODEL_FACTORIES, create_model_from_mst, dataset_of, pack_key,  # noqa: F401
                       register_model)
