<?php
echo "hello from php\n";
