#   Copyright IBM Corporation 2020
#
#   Licensed under the Apache License, Version 2.0 (the "License");
#   you may not use this file except in compliance with the License.
#   You may obtain a copy of the License at
#
#        http://www.apache.org/licenses/LICENSE-2.0
#
#   Unless required by applicable law or agreed to in writing, software
#   distributed under the License is distributed on an "AS IS" BASIS,
#   WITHOUT WARRANTIES OR CONDITIONS OF ANY KIND, either express or implied.
#   See the License for the specific language governing permissions and
#   limitations under the License.


cd containers/docker-compose/api/
./api-docker-build.sh
cd -
cd containers/docker-compose/
./docker-compose-docker-build.sh
cd -
cd containers/dockerfile/
./dockerfile-docker-build.sh
cd -
cd containers/golang/
./golang-docker-build.sh
cd -
cd containers/java-gradle/
./java-gradle-docker-build.sh
cd -
cd containers/java-maven/
./java-maven-docker-build.sh
cd -
cd containers/docker-compose/api/
./myproject-docker-compose-api-docker-build.sh
cd -
cd containers/docker-compose/web/
./myproject-docker-compose-web-docker-build.sh
cd -
cd containers/dockerfile/
./myproject-dockerfile-docker-build.sh
cd -
cd containers/nodejs/
./nodejs-docker-build.sh
cd -
cd containers/php/
./php-docker-build.sh
cd -
cd containers/python/
./python-docker-build.sh
cd -
cd containers/ruby/
./ruby-docker-build.sh
cd -
cd containers/docker-compose/web/
./web-docker-build.sh
cd -
