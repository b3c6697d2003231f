"""Model zoo: GPT-3 family, BERT, ResNet/vision models (re-exported from vision.models)."""
from .gpt import GPTConfig, GPTForPretraining, GPTModel, gpt_config, gpt_1_3b, gpt_pretraining_loss  # noqa: F401
from .gpt import GPTForPretrainingPipe, GPTEmbeddingPipe, GPTPretrainingCriterionPipe  # noqa: F401
from .bert import BertConfig, BertModel, BertForPretraining, BertPretrainingCriterion, bert_config  # noqa: F401,E402
