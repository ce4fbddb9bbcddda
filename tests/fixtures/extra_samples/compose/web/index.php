<?php echo "web\n";
